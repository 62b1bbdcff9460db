"""Multi-GPU frames, one process per GPU (torch.distributed over RCCL/xGMI): image rows +
gather, re-dealt between frames from the ranks' measured kernel times
(SURVEY.md §8(f) row 2). The C-ABI twin in one process is rt_multi (csrc/rt_multi.cpp).

The reference splits the image into contiguous row bands, one per Vulkan device, with the first
band taking the remainder (src/ray_trace.cpp:74-93), moves rows between devices from their
measured frame times (src/workload_tuner.hpp:38-104, fed at src/ray_trace.cpp:750-775, tearing
every Vulkan object down on each move) and never moves pixels between GPUs (each device presents
its own window, :96-105). Here the frame starts from row-exact interleaved strips (strip_rows: the
8-row strips of the full rounds dealt round robin, the rest as one contiguous run per rank, so
every rank holds floor(H / N) or ceil(H / N) rows), and one gather brings every rank's float4
accumulator rows to rank 0, where rt_scatter_rows puts them in place and rt_resolve_rgba8
tonemaps the whole image once (the rgba8 bytes are a function of the float sum, shader.rgen:65-66,
so they need not travel).

Balancing (`timer` given): before frame k every rank reads its own kernel time and per-row work
(the tile-cost record, rt_launch_row_weights) of frame k - lag — long finished, so no rank drains
its queue — and the ranks sum their per-row cost estimates over a CPU (gloo) group; every rank
then re-deals the same partition with rt_partition_rebalance (deterministic, so all ranks agree
without another message): band-end rows move from the slowest rank to the others. Only rows maps
change; the contexts, scenes and LPT records stay.

Pixels are independent and seeds are global (RT_SEED_GLOBAL), so the assembled image is
bit-identical to a one-GPU render whatever the world size or partition, in both random stream
modes. With the reference's per-pixel LCG stream (RT_RNG_PIXEL_STREAM) a pixel's samples are one
sequential chain, so a GPU holding 1/N of the pixels ends with its longest chain.
With the counter-based stream (RT_RNG_SAMPLE_HASH) the library splits each pixel's samples into
chunks spread over the lanes, so every GPU stays throughput-bound at any N.

The band renderer, assembler and timer are injectable so the same logic runs in CPU tests (gloo,
world size 2-3) with the oracle standing in for the GPU.
"""
from __future__ import annotations

from collections import deque
from typing import Callable, Optional

import numpy as np

STRIP = 8  # rows per strip: one 8x8 pixel tile high, the kernel's wave tile


def strip_rows(rank: int, world: int, height: int, strip: int = STRIP) -> np.ndarray:
    """Global rows of `rank` in the initial partition (rt_partition_strips, csrc/rt_plan.cpp): the
    rows of the floor(H / (strip * world)) full rounds as strips k = rank, rank + world, ... of
    `strip` rows, then run `rank` of the rest cut into `world` contiguous runs (the first
    rest % world one row longer)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    y0 = (height // (strip * world)) * strip * world
    rows = [y for k in range(rank, y0 // strip, world) for y in range(k * strip, (k + 1) * strip)]
    rest = height - y0
    base, extra = divmod(rest, world)
    start = y0 + rank * base + min(rank, extra)
    rows += list(range(start, start + base + (1 if rank < extra else 0)))
    return np.asarray(rows, np.int32)


def max_rows(world: int, height: int, strip: int = STRIP) -> int:
    return max(len(strip_rows(r, world, height, strip)) for r in range(world))


def row_costs(rows: np.ndarray, ms: float, weights: Optional[np.ndarray]) -> np.ndarray:
    """This rank's per-row cost estimates of one measured frame (csrc/rt_plan.cpp update_costs):
    the kernel time split over the band's rows in proportion to their tile-cost weights (each
    floored at 1 % of the mean), or evenly without weights."""
    n = len(rows)
    if n == 0 or not (ms > 0.0) or not np.isfinite(ms):
        return np.zeros(n)
    if weights is not None and len(weights) == n:
        w = np.where(np.isfinite(weights), weights, 0.0)
        sw = float(np.where(w > 0, w, 0.0).sum())
        if sw > 0.0:
            floor_w = 0.01 * sw / n
            wf = np.maximum(w, floor_w)
            return ms * wf / wf.sum()
    return np.full(n, ms / n)


def blend_costs(old: np.ndarray, new: np.ndarray, blend: float) -> np.ndarray:
    """Rows measured in `new` (> 0) take blend x the new estimate + (1 - blend) x their previous
    one (csrc/rt_plan.cpp update_costs): per-frame kernel times vary by a few tenths of a
    percent, which a re-deal should not chase."""
    out = old.copy()
    m = new > 0
    keep = (old > 0) & m & (blend < 1.0)
    out[m] = new[m]
    out[keep] = (1.0 - blend) * old[keep] + blend * new[keep]
    return out


class DistributedRenderer:
    """One rank's share of a multi-GPU frame.

    render_band(rows_dev, accum_dev, out_dev): renders this rank's rows into [rows, W, 4] buffers
    (rows_dev None at one rank: the whole frame, no row map).
    assemble(band_accum, band_out, rows_dev, full_accum, full_out): rank-0 reorder of one rank's
    gathered band into the full image (band_out / full_out None when only accumulators travel).
    resolve(full_accum, full_out): rank-0 tonemap of the assembled accumulator; when given (with
    gather_accum), only the accumulators are gathered. Without it both images are gathered.
    force_gather: run the gather + reassembly even on one rank (tests of the collective path).
    timer(back, band_rows) -> (ms, weights | None): this rank's kernel time of its launch `back`
    launches before its most recent one, and that band's per-row work weights; given, the rows are
    re-dealt between frames (balance; tolerance / lag / blend as rt_multi's balancer).
    """

    def __init__(self, width: int, height: int, device, render_band: Callable,
                 assemble: Optional[Callable] = None, strip: int = STRIP, gather_accum: bool = True,
                 force_gather: bool = False, resolve: Optional[Callable] = None,
                 timer: Optional[Callable] = None, tolerance: float = 0.001, lag: int = 2,
                 blend: float = 0.5):
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
        self.strip = strip
        # one rank: the identity map is left out (no per-sample row lookup in the kernel)
        self.multi = self.world > 1 or force_gather
        # gloo moves host tensors only: stage device bands through host memory (rehearsal of the
        # multi-rank path on a shared GPU; RCCL gathers device memory directly).
        self.staged = (self.world > 1 and getattr(device, "type", str(device)) != "cpu"
                       and dist.get_backend() == "gloo")
        self.timer = timer if self.multi else None   # (one rank + force_gather: the exchange path runs, no move)
        if not (0.0 < blend <= 1.0):
            raise ValueError("blend must be in (0, 1]")
        self.tolerance, self.lag, self.blend = tolerance, max(1, int(lag)), blend
        self.cost = np.zeros(height, np.float64)
        self.history = deque()      # per frame: (partition, launch index of this rank or None)
        self.launches = 0           # render_band calls that launched (rows present)
        self.rebalances = 0
        self.rows_moved = 0
        self.predicted = 1.0
        self.cpu_group = None
        if self.timer is not None and dist.get_backend() != "gloo":
            # the per-row costs travel on the host: a device all-reduce would queue behind the
            # frame's persistent kernel and stall the host for it. Without a gloo group (it is a
            # collective call, so every rank sees the same outcome) the split stays static.
            try:
                self.cpu_group = dist.new_group(backend="gloo")
            except Exception as e:  # noqa: BLE001
                import sys
                print(f"rtvk.dist: no gloo group ({e}); row split static", file=sys.stderr)
                self.timer = None
        self.cap = 0
        self._set_parts([strip_rows(r, self.world, height, strip) for r in range(self.world)])

    # ---- partition ------------------------------------------------------------------------
    def _set_parts(self, parts):
        torch = self.torch
        self.parts = [np.asarray(p, np.int32) for p in parts]
        self.rows_np = self.parts[self.rank]
        self.n = len(self.rows_np)
        self.nmax = max(len(p) for p in self.parts)
        self.rows = torch.from_numpy(self.rows_np.copy()).to(self.device) if self.multi else None
        if self.nmax > self.cap:
            # bands are padded to a common capacity so one fixed-size gather moves every rank's rows;
            # room for a few moved rows so a re-deal rarely reallocates (same on every rank)
            self.cap = min(self.H, self.nmax + (self.strip if self.world > 1 else 0))
            self.accum = torch.zeros((self.cap, self.W, 4), dtype=torch.float32, device=self.device)
            self.out = torch.zeros((self.cap, self.W, 4), dtype=torch.uint8, device=self.device)
            if self.rank == 0 and self.multi:
                self.g_accum = [torch.empty_like(self.accum) for _ in range(self.world)]
                self.g_out = [torch.empty_like(self.out) for _ in range(self.world)] if self.resolve is None else None
        if self.rank == 0 and self.multi:
            self.all_rows = [torch.from_numpy(p.copy()).to(self.device) for p in self.parts]
            if not hasattr(self, "full_accum"):
                self.full_accum = torch.zeros((self.H, self.W, 4), dtype=torch.float32, device=self.device)
                self.full_out = torch.zeros((self.H, self.W, 4), dtype=torch.uint8, device=self.device)

    def rows_per_rank(self) -> list:
        return [len(p) for p in self.parts]

    def _balance(self):
        """Re-deal from frame k - lag (every rank calls it at the same frame)."""
        if self.timer is None or len(self.history) < self.lag:
            return
        parts_m, launch = self.history[-self.lag]
        mine = np.zeros(self.H, np.float64)
        if launch is not None:
            rows = parts_m[self.rank]
            ms, w = self.timer(self.launches - 1 - launch, len(rows))
            mine[rows] = row_costs(rows, ms, w)
        t = self.torch.from_numpy(mine)
        self.dist.all_reduce(t, group=self.cpu_group)   # disjoint rows: the sum is every rank's estimate
        self.cost = blend_costs(self.cost, t.numpy(), self.blend)
        from . import partition_rebalance
        parts, moved, pred = partition_rebalance(self.parts, self.cost, tolerance=self.tolerance)
        if moved:
            self.rebalances += 1
            self.rows_moved += moved
            self.predicted = pred
            self._set_parts(parts)

    # ---- one frame -----------------------------------------------------------------------
    def step(self):
        """Render this rank's rows, gather to rank 0, assemble. Returns (accum, rgba8) of the
        full image on rank 0, None elsewhere."""
        self._balance()
        self.render_band(self.rows, self.accum[: self.n], self.out[: self.n])
        launch = None
        if self.n:
            launch = self.launches
            self.launches += 1
        self.history.append(([p.copy() for p in self.parts], launch))
        while len(self.history) > max(4, self.lag + 1):
            self.history.popleft()
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


def hip_band_timer(renderer):
    """timer backed by the library's per-launch records: rt_launch_ms (HIP events around the trace
    kernel) and rt_launch_row_weights (the launch's tile-cost record); both wait for that launch
    only."""
    def timer(back, band_rows):
        ms = renderer.launch_ms(back)
        try:
            w = renderer.launch_row_weights(band_rows, back)
        except Exception:
            w = None   # no record kept (brute force): the time alone
        return ms, w
    return timer


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
