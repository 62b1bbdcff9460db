"""rtvk — host-side mirror of the reference's hot-path API over librt_mi355x.so.

Names follow the reference:
  generateRandomScene(t)           src/scene.h:79-157 (t explicit instead of the wall clock)
  RenderCallInfo / Sphere / Scene  src/render_call_info.h:5-13, src/scene.h:16-29
  ray_trace(samples, storeRenderResult, width, height, gpu_count)
                                   src/ray_trace.h:9-15 (headless; renders once and returns)
and the per-frame device work of src/ray_trace.cpp:567-739 is ``Renderer.render_device``.

Everything computes in the HIP library; this module only marshals arguments. Device buffers are
torch tensors (memory + stream plumbing only).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Iterable, Optional, Sequence

import numpy as np

from . import abi
from .abi import (CHECKERED, DIFFUSE, METAL, REFRACTIVE, SOLID, Options, RenderCallInfo, RtError,
                  Scene, Sphere, Stats, check, load_library)

__all__ = [
    "DIFFUSE", "METAL", "REFRACTIVE", "SOLID", "CHECKERED", "Sphere", "Scene", "RenderCallInfo",
    "Options", "Stats", "RtError", "generateRandomScene", "canonical_render_call_info",
    "make_options", "Renderer", "MultiRenderer", "render", "ray_trace", "store_ppm", "spheres_to_numpy",
    "load_library", "HASH", "STREAM", "multi_plan", "partition_strips", "partition_rebalance",
]

STREAM = abi.RT_RNG_PIXEL_STREAM   # the reference's per-pixel LCG stream (random.glsl)
HASH = abi.RT_RNG_SAMPLE_HASH      # counter-based per-sample streams, chunked across lanes / GPUs

MAX_DEPTH = 50  # shader.rgen:27


def generateRandomScene(t: float = 0.0, grid_half_extent: int = 11):
    """src/scene.h:79-157: ground + 3 big spheres + (2K)^2 grid; K = 11 gives the 488-sphere scene.

    Returns a ctypes array of ``Sphere`` (length 4 + 4K^2)."""
    lib = load_library()
    n = ctypes.c_uint32()
    check(lib.rt_generate_scene(ctypes.c_float(t), grid_half_extent, None, 0, ctypes.byref(n)))
    arr = (Sphere * n.value)()
    check(lib.rt_generate_scene(ctypes.c_float(t), grid_half_extent, ctypes.addressof(arr), n.value,
                                ctypes.byref(n)))
    return arr


def spheres_to_numpy(spheres) -> np.ndarray:
    """Raw 80-byte records as a (n, 80) uint8 array (for hashing / fixtures)."""
    return np.frombuffer(bytes(spheres), dtype=np.uint8).reshape(-1, 80)


def canonical_render_call_info(spp: int, width: int = 1920, height: int = 1080) -> RenderCallInfo:
    """The RenderCallInfo the reference fills every frame (src/ray_trace.cpp:660-676)."""
    rci = RenderCallInfo()
    check(load_library().rt_canonical_render_call_info(spp, width, height, ctypes.byref(rci)))
    return rci


def make_options(max_depth: int = MAX_DEPTH, seed_mode: int = abi.RT_SEED_GLOBAL,
                 rng_mode: int = abi.RT_RNG_PIXEL_STREAM, accel: int = abi.RT_ACCEL_AUTO,
                 accumulate: bool = False, sample_base: int = 0, count_tests: bool = False) -> Options:
    o = Options()
    o.max_depth, o.seed_mode, o.rng_mode, o.accel = max_depth, seed_mode, rng_mode, accel
    o.accumulate, o.sample_base = int(bool(accumulate)), sample_base
    o.reserved[0] = 1 if count_tests else 0
    return o


def _stream_ptr(stream, device: int) -> Optional[int]:
    """hipStream_t of `stream`, or of torch's current stream ON `device` when None (torch's
    current device may be another GPU)."""
    if stream is None:
        import torch
        return torch.cuda.current_stream(device).cuda_stream
    return getattr(stream, "cuda_stream", stream)


def _check_dev_tensor(t, dtype_name: str, shape: Sequence[int]):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError("expected a device (cuda) torch.Tensor")
    if str(t.dtype) != dtype_name or not t.is_contiguous() or tuple(t.shape) != tuple(shape):
        raise ValueError(f"expected contiguous {dtype_name} tensor of shape {tuple(shape)}, "
                         f"got {t.dtype} {tuple(t.shape)}")


class Renderer:
    """One device context: HBM-resident scene + LBVH, and the fused trace kernel.

    Replaces, per GPU, the reference's descriptor set / BLAS / TLAS / pipeline
    (src/ray_trace.cpp:315-527) and its per-frame command buffer (src/vulkan.h:998-1204)."""

    def __init__(self, device: int = 0):
        self._lib = load_library()
        self._ctx = ctypes.c_void_p()
        check(self._lib.rt_context_create(device, ctypes.byref(self._ctx)))
        self.device = device
        self.sphere_count = 0

    def close(self) -> None:
        if self._ctx:
            self._lib.rt_context_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, spheres, stream=None) -> None:
        """Upload spheres (ctypes Sphere array or (n,80) uint8 records) and build the LBVH, ordered
        on `stream` (torch's current stream by default, like render_device)."""
        buf = spheres if not isinstance(spheres, np.ndarray) else np.ascontiguousarray(spheres, np.uint8)
        n = len(spheres)
        ptr = ctypes.addressof(buf) if not isinstance(buf, np.ndarray) else buf.ctypes.data
        st = _stream_ptr(stream, self.device)
        check(self._lib.rt_set_scene(self._ctx, ptr if n else None, n, st))
        self.sphere_count = n

    def refit_scene(self, spheres, stream=None) -> None:
        """Per-frame update (same count): refit the device-built tree to moved spheres."""
        buf = spheres if not isinstance(spheres, np.ndarray) else np.ascontiguousarray(spheres, np.uint8)
        n = len(spheres)
        ptr = ctypes.addressof(buf) if not isinstance(buf, np.ndarray) else buf.ctypes.data
        st = _stream_ptr(stream, self.device)
        check(self._lib.rt_refit_scene(self._ctx, ptr if n else None, n, st))
        self.sphere_count = n

    def set_scene_device(self, spheres_dev, refit: bool = False, stream=None) -> None:
        """Spheres already on the device: a contiguous uint8 cuda tensor [n, 80]."""
        import torch
        if not spheres_dev.is_cuda or spheres_dev.dtype != torch.uint8 or spheres_dev.dim() != 2 \
                or spheres_dev.shape[1] != 80 or not spheres_dev.is_contiguous():
            raise ValueError("spheres_dev must be a contiguous uint8 cuda tensor [n, 80]")
        n = int(spheres_dev.shape[0])
        st = _stream_ptr(stream, self.device)
        fn = self._lib.rt_refit_scene_device if refit else self._lib.rt_set_scene_device
        check(fn(self._ctx, spheres_dev.data_ptr() if n else None, n, st))
        self.sphere_count = n

    def tune(self, **kv) -> None:
        """Launch-plan parameters of this context (rt_debug_tune; tests and A/B timing only): e.g.
        ``tune(sample_chunks=7)``; None restores a default. No setting changes an image."""
        for k, v in kv.items():
            check(self._lib.rt_debug_tune(self._ctx, k.encode(), -1.0 if v is None else float(v)))

    def tile_costs(self) -> np.ndarray:
        """Per 8x8 tile of the last LBVH launch, the traced segments of its most expensive pixel
        (row-major tiles; empty before the first launch): the key the next launch hands tiles out
        by, longest first."""
        n = ctypes.c_uint64(0)
        check(self._lib.rt_debug_tile_cost(self._ctx, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, np.uint32)
        if n.value:
            check(self._lib.rt_debug_tile_cost(self._ctx, out.ctypes.data, n.value, ctypes.byref(n)))
        return out

    _SCENE_DTYPES = {0: (np.float32, 4), 1: (np.float32, 1), 2: (np.uint8, 32), 3: (np.uint32, 1),
                     4: (np.uint8, 32), 5: (np.uint8, 32), 6: (np.float32, 4), 7: (np.uint32, 1)}

    def scene_array(self, what: int) -> np.ndarray:
        """Diagnostic copy of one device scene array (rt_debug_scene); what 8 (scene) and 9 (grid
        layout) return a dict."""
        nbytes = ctypes.c_uint64(0)
        if what == 9:
            g = (ctypes.c_uint32 * 5)()
            check(self._lib.rt_debug_scene(self._ctx, 9, g, 20, ctypes.byref(nbytes)))
            return {"n": (int(g[0]), int(g[1]), int(g[2])), "cells": int(g[3]), "refs": int(g[4])}
        if what == 8:
            raw = (ctypes.c_uint8 * 32)()
            check(self._lib.rt_debug_scene(self._ctx, 8, raw, 32, ctypes.byref(nbytes)))
            u = np.frombuffer(bytes(raw), np.uint32)
            f = np.frombuffer(bytes(raw), np.float32)
            return {"n_spheres": int(u[0]), "n_big": int(u[1]), "n_nodes": int(u[2]),
                    "n_leaf": int(u[3]), "device_built": bool(u[4]), "small_rmax": float(f[6]),
                    "scene_radius": float(f[7])}
        self._lib.rt_debug_scene(self._ctx, what, None, 0, ctypes.byref(nbytes))   # size query
        buf = np.zeros(max(1, nbytes.value), np.uint8)
        if nbytes.value:
            check(self._lib.rt_debug_scene(self._ctx, what, buf.ctypes.data, nbytes.value, ctypes.byref(nbytes)))
        dt, w = self._SCENE_DTYPES[what]
        a = buf[: nbytes.value].view(dt)
        return a.reshape(-1, w) if w > 1 else a

    def render_device(self, rci: RenderCallInfo, accum, out, rows=None,
                      options: Optional[Options] = None, stream=None) -> None:
        """One band on this device, asynchronous on `stream` (torch current stream by default).

        accum: float32 cuda tensor [band_h, band_w, 4]; out: uint8 cuda tensor [band_h, band_w, 4];
        rows: optional int32/uint32 cuda tensor [band_h] of global row indices (strip tiling)."""
        bh, bw = int(accum.shape[0]), int(accum.shape[1])
        _check_dev_tensor(accum, "torch.float32", (bh, bw, 4))
        _check_dev_tensor(out, "torch.uint8", (bh, bw, 4))
        rows_ptr = None
        if rows is not None:
            if rows.numel() != bh or not rows.is_cuda or rows.element_size() != 4 or not rows.is_contiguous():
                raise ValueError("rows must be a contiguous 4-byte cuda tensor of band_h entries")
            rows_ptr = rows.data_ptr()
        check(self._lib.rt_render_device(self._ctx, ctypes.byref(rci), rows_ptr, bw, bh,
                                         accum.data_ptr(), out.data_ptr(),
                                         ctypes.byref(options) if options is not None else None,
                                         _stream_ptr(stream, self.device)))

    def stats(self) -> Stats:
        st = Stats()
        check(self._lib.rt_get_stats(self._ctx, ctypes.byref(st)))
        return st

    def steals(self) -> int:
        """Tail steals of the last instrumented launch (count_tests; rt_debug_steals; counter-based
        stream only)."""
        v = ctypes.c_uint64()
        check(self._lib.rt_debug_steals(self._ctx, ctypes.byref(v)))
        return int(v.value)

    def grid_cells(self) -> dict:
        """Of the last instrumented (count_tests) grid-walk launch: cells visited and visited cells
        without references (rt_debug_grid_cells)."""
        v = (ctypes.c_uint64 * 2)()
        check(self._lib.rt_debug_grid_cells(self._ctx, v))
        return {"cells": int(v[0]), "empty": int(v[1])}

    def launch_info(self) -> dict:
        """Of the last launch: sample chunks per pixel (of the LPT order's tail ranks; head_chunks:
        of its head ranks, None when there is no head), the kernel form it ran, its dynamic LDS
        bytes, the CU count, whether its grid walk was the one-layer form (flat_grid: the grid is
        one cell thick in y) and whether its camera rays started at the camera position itself
        (pinhole_origin) (rt_debug_launch_info)."""
        v = (ctypes.c_uint32 * 4)()
        check(self._lib.rt_debug_launch_info(self._ctx, v))
        forms = {1: "brute", 2: "lbvh-global", 3: "lbvh-lds", 4: "lbvh-octant-lds", 5: "lbvh-treelet", 6: "grid-lds", 7: "grid-global",
                 8: "grid-lds-coop", 9: "grid-global-coop", 10: "grid-lds-rec", 11: "grid-lds-cq", 12: "grid-lds-rec-cq"}
        return {"chunks": int(v[0]) & 0xffff, "head_chunks": (int(v[0]) >> 16) or None,
                "form": forms.get(int(v[1]) & 0xffff, str(v[1])), "lds_bytes": int(v[2]), "cus": int(v[3]),
                "flat_grid": bool((int(v[1]) >> 16) & 1), "pinhole_origin": bool((int(v[1]) >> 17) & 1)}

    def scatter_rows(self, src_accum, src_rgba8, rows, dst_accum, dst_rgba8, stream=None) -> None:
        """dst[rows[i]] = src[i] (device), the reorder after a multi-GPU gather; either image may
        be None (both its source and destination)."""
        src = src_rgba8 if src_rgba8 is not None else src_accum
        dst = dst_rgba8 if dst_rgba8 is not None else dst_accum
        if src is None or dst is None:
            raise ValueError("nothing to scatter")
        n, w, dh = int(src.shape[0]), int(src.shape[1]), int(dst.shape[0])
        if (src_rgba8 is None) != (dst_rgba8 is None) or (src_accum is None) != (dst_accum is None):
            raise ValueError("each image needs both a source and a destination, or neither")
        if src_rgba8 is not None:
            _check_dev_tensor(src_rgba8, "torch.uint8", (n, w, 4))
            _check_dev_tensor(dst_rgba8, "torch.uint8", (dh, w, 4))
        if src_accum is not None:
            _check_dev_tensor(src_accum, "torch.float32", (n, w, 4))
            _check_dev_tensor(dst_accum, "torch.float32", (dh, w, 4))
        self._check_rows(rows, n, dh)
        check(self._lib.rt_scatter_rows(self._ctx, src_accum.data_ptr() if src_accum is not None else None,
                                        src_rgba8.data_ptr() if src_rgba8 is not None else None,
                                        rows.data_ptr(), n, w, dh,
                                        dst_accum.data_ptr() if dst_accum is not None else None,
                                        dst_rgba8.data_ptr() if dst_rgba8 is not None else None,
                                        _stream_ptr(stream, self.device)))

    @staticmethod
    def _check_rows(rows, n, limit):
        if rows.numel() != n or not rows.is_cuda or rows.element_size() != 4 or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous 4-byte cuda tensor of one entry per band row")
        if n and (int(rows.min()) < 0 or int(rows.max()) >= limit):
            raise ValueError(f"rows must lie in [0, {limit})")

    def gather_rows(self, src_accum, rows, dst_accum, stream=None) -> None:
        """dst[i] = src[rows[i]] (device float4 accumulators), the inverse of scatter_rows."""
        sh, w = int(src_accum.shape[0]), int(src_accum.shape[1])
        n = int(dst_accum.shape[0])
        _check_dev_tensor(src_accum, "torch.float32", (sh, w, 4))
        _check_dev_tensor(dst_accum, "torch.float32", (n, w, 4))
        self._check_rows(rows, n, sh)
        check(self._lib.rt_gather_rows(self._ctx, src_accum.data_ptr(), rows.data_ptr(), n, w, sh,
                                       dst_accum.data_ptr(), _stream_ptr(stream, self.device)))

    def resolve_rgba8(self, accum, spp: int, out, stream=None) -> None:
        """out = rgba8 tonemap of the summed float4 accumulator `accum` (device tensors), exactly
        as the trace kernel stores a pixel (rt_resolve_rgba8)."""
        n = accum.numel() // 4
        if out.numel() != 4 * n:
            raise ValueError("out must hold 4 bytes per accumulator texel")
        check(self._lib.rt_resolve_rgba8(self._ctx, accum.data_ptr(), n, spp, out.data_ptr(),
                                         _stream_ptr(stream, self.device)))

    def launch_ms(self, back: int = 0) -> float:
        """Trace-kernel ms of the launch `back` launches before the most recent one (rt_launch_ms:
        waits for that launch only, not for the ones queued after it)."""
        v = ctypes.c_float()
        check(self._lib.rt_launch_ms(self._ctx, back, ctypes.byref(v)))
        return float(v.value)

    def launch_row_weights(self, band_rows: int, back: int = 0) -> np.ndarray:
        """Per band row of the launch `back` launches before the most recent one, its share of the
        launch's work from the tile-cost record (rt_launch_row_weights; ratios only)."""
        w = np.zeros(max(1, band_rows), np.float64)
        check(self._lib.rt_launch_row_weights(self._ctx, back, w.ctypes.data, band_rows))
        return w[:band_rows]

    def kernel_times(self, n: int = 64) -> list:
        """Trace-kernel durations (ms) of the last `n` launches (at most 64 kept), oldest first:
        HIP events recorded around the kernel on its launch stream (rt_debug_kernel_times)."""
        buf = (ctypes.c_float * max(1, n))()
        got = ctypes.c_uint32(0)
        check(self._lib.rt_debug_kernel_times(self._ctx, buf, n, ctypes.byref(got)))
        return [float(buf[i]) for i in range(got.value)]


class MultiRenderer:
    """One process driving `gpu_count` GPUs (rt_multi): one context + stream per device and one
    RCCL communicator over them. A frame tiles the image into row-exact interleaved strips
    (partition_strips), re-dealt between frames from the devices' measured kernel times, and
    gathers every device's rows to device 0 over xGMI (grouped ncclSend / ncclRecv), where they
    are reordered; the image equals the one-GPU image bit for bit.

    logical=True (tests on a one-GPU box): `gpu_count` logical devices on GPU 0 running the same
    frame plans, each RCCL send / receive pair a device copy (rt_debug_multi_create_logical), or
    with logical="rccl" RCCL send / receive of a one-rank communicator to itself
    (rt_debug_multi_create_logical_rccl)."""

    def __init__(self, gpu_count: int = 1, logical=False):
        self._lib = load_library()
        self._m = ctypes.c_void_p()
        create = (self._lib.rt_debug_multi_create_logical_rccl if logical == "rccl"
                  else self._lib.rt_debug_multi_create_logical if logical else self._lib.rt_multi_create)
        check(create(gpu_count, ctypes.byref(self._m)))
        n = ctypes.c_uint32()
        check(self._lib.rt_multi_device_count(self._m, ctypes.byref(n)))
        self.device_count = n.value

    def close(self) -> None:
        if self._m:
            self._lib.rt_multi_destroy(self._m)
            self._m = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, spheres) -> None:
        buf = spheres if not isinstance(spheres, np.ndarray) else np.ascontiguousarray(spheres, np.uint8)
        ptr = ctypes.addressof(buf) if not isinstance(buf, np.ndarray) else buf.ctypes.data
        check(self._lib.rt_multi_set_scene(self._m, ptr if len(spheres) else None, len(spheres)))

    def render(self, rci: RenderCallInfo, accum, out, options: Optional[Options] = None, stream=None) -> None:
        """One frame into device-0 tensors accum (float32 [H, W, 4]) and out (uint8 [H, W, 4])."""
        W, H = rci.image_size.x, rci.image_size.y
        _check_dev_tensor(accum, "torch.float32", (H, W, 4))
        _check_dev_tensor(out, "torch.uint8", (H, W, 4))
        if accum.device.index != 0 or out.device.index != 0:
            raise ValueError("MultiRenderer.render gathers to device 0: accum and out must live on cuda:0")
        check(self._lib.rt_multi_render(self._m, ctypes.byref(rci),
                                        ctypes.byref(options) if options is not None else None,
                                        accum.data_ptr(), out.data_ptr(), _stream_ptr(stream, 0)))

    def info(self) -> dict:
        """{devices, rccl_ranks (ncclCommCount of the communicator), strip_rows, launches of the
        last frame} (rt_multi_info)."""
        v = (ctypes.c_uint32 * 4)()
        check(self._lib.rt_multi_info(self._m, v))
        return {"devices": int(v[0]), "rccl_ranks": int(v[1]), "strip_rows": int(v[2]), "launches": int(v[3])}

    def kernel_times(self, frames: Optional[int] = None) -> list:
        """Trace-kernel ms of the last frame on each device that rendered rows (device order); with
        `frames`, a list of such lists for each of the last `frames` frames, oldest first."""
        if frames is None:
            buf = (ctypes.c_float * max(1, self.device_count))()
            got = ctypes.c_uint32(0)
            check(self._lib.rt_multi_kernel_times(self._m, buf, self.device_count, ctypes.byref(got)))
            return [float(buf[i]) for i in range(got.value)]
        cap = frames * self.device_count
        buf = (ctypes.c_float * max(1, cap))()
        got = ctypes.c_uint32(0)
        check(self._lib.rt_multi_kernel_times_frames(self._m, frames, buf, cap, ctypes.byref(got)))
        n = got.value // max(1, frames)
        return [[float(buf[f * n + d]) for d in range(n)] for f in range(frames)]

    def stats(self) -> Stats:
        st = Stats()
        check(self._lib.rt_multi_stats(self._m, ctypes.byref(st)))
        return st

    def partition(self, height: int) -> list:
        """The rows each device renders in the next frame (band order), one uint32 array per
        device (rt_multi_partition)."""
        counts = np.zeros(self.device_count, np.uint32)
        rows = np.zeros(max(1, height), np.uint32)
        check(self._lib.rt_multi_partition(self._m, rows.ctypes.data, counts.ctypes.data, height))
        return _split(rows, counts)

    def tune(self, **kv) -> None:
        """Balancer settings (rt_debug_multi_tune): balance=0/1, tolerance, blend in (0, 1], lag 1-8;
        None restores a default."""
        for k, v in kv.items():
            check(self._lib.rt_debug_multi_tune(self._m, k.encode(), -1.0 if v is None else float(v)))

    def feedback(self, device_ms: Sequence[float]) -> None:
        """Device times the next frame re-deals from, as if measured (rt_debug_multi_feedback)."""
        buf = (ctypes.c_float * max(1, len(device_ms)))(*device_ms)
        check(self._lib.rt_debug_multi_feedback(self._m, buf, len(device_ms)))

    def balance_info(self) -> dict:
        v = (ctypes.c_double * 4)()
        check(self._lib.rt_debug_multi_balance_info(self._m, v))
        return {"frames": int(v[0]), "rebalances": int(v[1]), "rows_moved": int(v[2]),
                "predicted_imbalance": float(v[3])}


def _split(rows: np.ndarray, counts: np.ndarray) -> list:
    out, at = [], 0
    for c in counts:
        out.append(rows[at:at + int(c)].copy())
        at += int(c)
    return out


def _flat(parts: Sequence) -> tuple:
    counts = np.asarray([len(p) for p in parts], np.uint32)
    rows = np.ascontiguousarray(np.concatenate([np.asarray(p, np.uint32) for p in parts])
                                if len(parts) else np.zeros(0, np.uint32), np.uint32)
    return rows, counts


def partition_strips(n_devices: int, height: int) -> list:
    """The row-exact interleaved strips every multi-device frame starts from (rt_partition_strips):
    one uint32 array of global rows per device, band order."""
    counts = np.zeros(n_devices, np.uint32)
    rows = np.zeros(max(1, height), np.uint32)
    check(load_library().rt_partition_strips(n_devices, height, rows.ctypes.data, counts.ctypes.data))
    return _split(rows, counts)


def partition_rebalance(parts: Sequence, cost: np.ndarray, measured: Optional[Sequence] = None,
                        device_ms: Optional[Sequence[float]] = None, tolerance: float = 0.001) -> tuple:
    """One balancing step (rt_partition_rebalance): rescale the per-row costs `cost` (float64 [H],
    <= 0 unknown; updated in place) to the device times `device_ms` measured on partition
    `measured`, then re-deal `parts`. Returns (new parts, rows moved, predicted max / mean)."""
    lib = load_library()
    n, H = len(parts), int(cost.shape[0])
    if cost.dtype != np.float64 or not cost.flags.c_contiguous:
        raise ValueError("cost must be a contiguous float64 array")
    rows, counts = _flat(parts)
    if len(rows) != H:
        raise ValueError("the partition must hold every row exactly once")
    m_rows = m_counts = m_ms = None
    keep = []
    if measured is not None:
        mr, mc = _flat(measured)
        ms = np.ascontiguousarray(np.asarray(device_ms, np.float32))
        if len(ms) != n or len(mc) != n:
            raise ValueError("one measured time per device")
        keep = [mr, mc, ms]
        m_rows, m_counts, m_ms = mr.ctypes.data, mc.ctypes.data, ms.ctypes.data
    moved = ctypes.c_uint32(0)
    pred = ctypes.c_double(1.0)
    check(lib.rt_partition_rebalance(n, H, rows.ctypes.data, counts.ctypes.data, cost.ctypes.data, m_rows, m_counts,
                                     m_ms, float(tolerance), ctypes.byref(moved), ctypes.byref(pred)))
    del keep
    return _split(rows, counts), int(moved.value), float(pred.value)


PLAN_OPS = {1: "load_rows", 2: "group_start", 3: "send", 4: "recv", 5: "group_end", 6: "render",
            7: "store_rows", 8: "resolve"}


def multi_plan(n_devices: int, width: int, height: int, band_starts: Optional[Sequence[int]] = None,
               accumulate: bool = False, parts: Optional[Sequence] = None) -> dict:
    """The frame plan rt_multi executes (rt_debug_multi_plan; host only, no GPU needed): the parts
    [(device, whole, rows)] and the ordered steps [{op, dev, peer, part, flags, count}]. band_starts
    None: the row-exact strips (rt_multi_render's first frame); else the bands of rt_render; parts:
    an explicit partition (one row array per device, e.g. a re-dealt one; rt_debug_multi_plan_rows)."""
    lib = load_library()
    n = ctypes.c_uint64(0)
    if parts is not None:
        rows, counts = _flat(parts)
        if len(counts) != n_devices:
            raise ValueError("one row array per device")
        call = lambda out, cap: lib.rt_debug_multi_plan_rows(n_devices, width, height, rows.ctypes.data,  # noqa: E731
                                                              counts.ctypes.data, int(accumulate), out, cap,
                                                              ctypes.byref(n))
    else:
        bs = None if band_starts is None else (ctypes.c_uint32 * len(band_starts))(*band_starts)
        nb = 0 if band_starts is None else len(band_starts)
        call = lambda out, cap: lib.rt_debug_multi_plan(n_devices, width, height, bs, nb, int(accumulate),  # noqa: E731
                                                         out, cap, ctypes.byref(n))
    check(call(None, 0))
    buf = np.zeros(n.value, np.uint32)
    check(call(buf.ctypes.data, n.value))
    n_parts, n_steps = int(buf[0]), int(buf[1])
    at, parts, steps = 2, [], []
    for _ in range(n_parts):
        dev, whole, nr = (int(v) for v in buf[at:at + 3])
        parts.append((dev, bool(whole), buf[at + 3:at + 3 + nr].copy()))
        at += 3 + nr
    for _ in range(n_steps):
        op, dev, peer, part, flags, lo, hi = (int(v) for v in buf[at:at + 7])
        steps.append({"op": PLAN_OPS.get(op, op), "dev": dev, "peer": peer, "part": part, "flags": flags,
                      "count": lo | (hi << 32)})
        at += 7
    assert at == len(buf)
    return {"parts": parts, "steps": steps}


@dataclass
class RenderResult:
    accum: np.ndarray   # float32 [H, W, 4] — the rgba32f sum image (binding 3)
    rgba8: np.ndarray   # uint8   [H, W, 4] — the tonemapped image (binding 0)
    stats: Stats


def render(spheres, rci: RenderCallInfo | Sequence[RenderCallInfo], options: Optional[Options] = None,
           accum: Optional[np.ndarray] = None) -> RenderResult:
    """Host-buffer frame (rt_render): one band per RenderCallInfo, band i on device i % ndev."""
    lib = load_library()
    rcis = [rci] if isinstance(rci, RenderCallInfo) else list(rci)
    arr = (RenderCallInfo * len(rcis))(*rcis)
    W, H = rcis[0].image_size.x, rcis[0].image_size.y
    acc = np.zeros((H, W, 4), np.float32) if accum is None else np.ascontiguousarray(accum, np.float32)
    out = np.zeros((H, W, 4), np.uint8)
    st = Stats()
    sp = spheres if not isinstance(spheres, np.ndarray) else np.ascontiguousarray(spheres, np.uint8)
    sptr = ctypes.addressof(sp) if not isinstance(sp, np.ndarray) else sp.ctypes.data
    check(lib.rt_render(sptr, len(spheres), ctypes.addressof(arr), len(rcis), acc.ctypes.data,
                        out.ctypes.data, ctypes.byref(options) if options is not None else None,
                        ctypes.byref(st)))
    return RenderResult(acc, out, st)


def store_ppm(path: str, rgba8: np.ndarray) -> None:
    h, w = rgba8.shape[:2]
    img = np.ascontiguousarray(rgba8, np.uint8)
    check(load_library().rt_store_ppm(str(path).encode(), img.ctypes.data, w, h))


def ray_trace(samples: int = 10, storeRenderResult: bool = False, width: int = 1920,
              height: int = 1080, gpu_count: int = 1) -> None:
    """src/ray_trace.h:9-15, same parameters and defaults (the C symbol, called through ctypes)."""
    load_library().ray_trace(samples, storeRenderResult, width, height, gpu_count)
