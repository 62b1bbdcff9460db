"""Multi-GPU frames, one process per GPU (torch.distributed over RCCL/xGMI): image strips +
gather. The C-ABI twin in one process is rt_multi (csrc/rt_multi.cpp).

The reference splits the image into contiguous row bands, one per Vulkan device, with the first
band taking the remainder (src/ray_trace.cpp:74-93), and never moves pixels between GPUs (each
device presents its own window, :96-105). Here rank r renders the 8-row strips k with
k % world == r — interleaving balances sky-heavy and sphere-heavy rows without the reference's
tuner (src/workload_tuner.hpp) — and one gather brings every rank's float4 accumulator strips to
rank 0, where rt_scatter_rows puts them in place and rt_resolve_rgba8 tonemaps the whole image
once (the rgba8 bytes are a function of the float sum, shader.rgen:65-66, so they need not
travel: 20 % fewer bytes and half the collectives of gathering both images).

Pixels are independent and seeds are global (RT_SEED_GLOBAL), so the assembled image is
bit-identical to a one-GPU render whatever the world size, in both random stream modes. With the
reference's per-pixel LCG stream (RT_RNG_PIXEL_STREAM) a pixel's samples are one sequential chain,
so a GPU holding 1/N of the pixels ends with its longest chain. With the
counter-based stream (RT_RNG_SAMPLE_HASH) the library splits each pixel's samples into chunks
spread over the lanes, so every GPU stays throughput-bound at any N.

The band renderer and the assembler are injectable so the same gather logic runs in CPU tests
(gloo, world size 2) with the oracle standing in for the GPU.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

STRIP = 8  # rows per strip: one 8x8 pixel tile high, the kernel's wave tile


def strip_rows(rank: int, world: int, height: int, strip: int = STRIP) -> np.ndarray:
    """Global rows of `rank`: strips k = rank, rank + world, ... of `strip` rows each."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    n_strips = (height + strip - 1) // strip
    rows = [y for k in range(rank, n_strips, world) for y in range(k * strip, min((k + 1) * strip, height))]
    return np.asarray(rows, np.int32)


def max_rows(world: int, height: int, strip: int = STRIP) -> int:
    return max(len(strip_rows(r, world, height, strip)) for r in range(world))


class DistributedRenderer:
    """One rank's share of a multi-GPU frame.

    render_band(rows_dev, accum_dev, out_dev): renders this rank's rows into [rows, W, 4] buffers
    (rows_dev None at one rank: the whole frame, no row map).
    assemble(band_accum, band_out, rows_dev, full_accum, full_out): rank-0 reorder of one rank's
    gathered band into the full image (band_out / full_out None when only accumulators travel).
    resolve(full_accum, full_out): rank-0 tonemap of the assembled accumulator; when given (with
    gather_accum), only the accumulators are gathered. Without it both images are gathered.
    force_gather: run the gather + reassembly even on one rank (tests of the collective path).
    """

    def __init__(self, width: int, height: int, device, render_band: Callable,
                 assemble: Optional[Callable] = None, strip: int = STRIP, gather_accum: bool = True,
                 force_gather: bool = False, resolve: Optional[Callable] = None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.W, self.H, self.device = width, height, device
        self.render_band = render_band
        self.assemble = assemble
        self.gather_accum = gather_accum
        self.resolve = resolve if gather_accum else None
        self.rows_np = strip_rows(self.rank, self.world, height, strip)
        self.nmax = max_rows(self.world, height, strip)
        n = len(self.rows_np)
        # Bands are padded to the largest band so one fixed-size gather moves every rank's rows.
        # one rank: the identity map is left out (no per-sample row lookup in the kernel)
        self.multi = self.world > 1 or force_gather
        self.rows = torch.from_numpy(self.rows_np).to(device) if self.multi else None
        self.accum = torch.zeros((self.nmax, width, 4), dtype=torch.float32, device=device)
        self.out = torch.zeros((self.nmax, width, 4), dtype=torch.uint8, device=device)
        self.n = n
        # gloo moves host tensors only: stage device bands through host memory (rehearsal of the
        # multi-rank path on a shared GPU; RCCL gathers device memory directly).
        self.staged = (self.world > 1 and getattr(device, "type", str(device)) != "cpu"
                       and dist.get_backend() == "gloo")
        if self.rank == 0 and self.multi:
            self.all_rows = [torch.from_numpy(strip_rows(r, self.world, height, strip)).to(device)
                             for r in range(self.world)]
            self.g_accum = [torch.empty_like(self.accum) for _ in range(self.world)]
            self.g_out = [torch.empty_like(self.out) for _ in range(self.world)] if resolve is None else None
            self.full_accum = torch.zeros((height, width, 4), dtype=torch.float32, device=device)
            self.full_out = torch.zeros((height, width, 4), dtype=torch.uint8, device=device)

    def step(self):
        """Render this rank's strips, gather to rank 0, assemble. Returns (accum, rgba8) of the
        full image on rank 0, None elsewhere."""
        self.render_band(self.rows, self.accum[: self.n], self.out[: self.n])
        if not self.multi:
            return self.accum[: self.n], self.out[: self.n]
        if self.gather_accum:
            self._gather(self.accum, self.g_accum if self.rank == 0 else None)
        if self.resolve is None:
            self._gather(self.out, self.g_out if self.rank == 0 else None)
        if self.rank != 0:
            return None
        for r in range(self.world):
            rows = self.all_rows[r]
            k = rows.numel()
            self.assemble(self.g_accum[r][:k] if self.gather_accum else None,
                          None if self.resolve is not None else self.g_out[r][:k], rows,
                          self.full_accum if self.gather_accum else None,
                          None if self.resolve is not None else self.full_out)
        if self.resolve is not None:
            self.resolve(self.full_accum, self.full_out)
        return self.full_accum, self.full_out

    def _gather(self, band, glist):
        dist = self.dist
        if not self.staged:
            dist.gather(band, glist, dst=0)
            return
        host = band.cpu()
        hlist = [self.torch.empty_like(host) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(host, hlist, dst=0)
        if self.rank == 0:
            for g, h in zip(glist, hlist):
                g.copy_(h)


def hip_band_renderer(renderer, rci, options, stream=None):
    """render_band backed by librt_mi355x.so (rt_render_device with a rows map)."""
    def render_band(rows, accum, out):
        if rows is None or rows.numel():
            renderer.render_device(rci, accum, out, rows=rows, options=options, stream=stream)
    return render_band


def hip_assembler(renderer, stream=None):
    """assemble backed by rt_scatter_rows (device kernel)."""
    def assemble(band_accum, band_out, rows, full_accum, full_out):
        if rows.numel():
            renderer.scatter_rows(band_accum, band_out, rows, full_accum, full_out, stream=stream)
    return assemble


def hip_resolver(renderer, spp: int, stream=None):
    """resolve backed by rt_resolve_rgba8 (device kernel, the trace kernel's own pixel store)."""
    def resolve(full_accum, full_out):
        renderer.resolve_rgba8(full_accum, spp, full_out, stream=stream)
    return resolve
