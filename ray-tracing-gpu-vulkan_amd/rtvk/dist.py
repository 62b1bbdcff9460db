"""Multi-GPU frames: sample split (default) or image strips, one process per GPU.

Sample split (SampleSplitRenderer). A pixel's samples form one sequential chain in the
reference's RNG (random.glsl: one LCG stream per pixel runs through every sample), so a GPU needs
several pixels per lane to hide the chain of its most expensive pixel: a 1080p/100-spp frame has
8 per lane on one MI355X, but only 1 per lane with 8-row strips on 8 GPUs, where the frame time is
the longest chain (~2000 segments) times the per-segment latency (measured: strips reach 0.9 /
0.5 / 0.3 of linear at 2 / 4 / 8 GPUs, scripts/scaling_probe.py). Instead, rank r renders the
whole frame with spp_r of the samples (sum spp_r = spp) and its own stream salt
RenderCallInfo.number + r (the reference's `number`, src/render_call_info.h:6, which exists to
decorrelate frames). Every GPU keeps all pixels and short chains; the accumulators are reduced by
an all-to-all of row slices, each rank adding the N slices of its part in rank order
(deterministic, so the frame equals the sum in rank order of N single-GPU frames with number =
r, alpha 1), then the slices are tonemapped (rt_reduce_resolve, fused with the sum) and gathered
to rank 0. With one GPU it is
exactly the reference frame.

Strips (DistributedRenderer): rank r renders the 8-row strips k = r mod N of the one-GPU frame
(bit-identical to it), gathered to rank 0. Kept for the reference-stream image at any N.

The reference splits the image into contiguous row bands, one per Vulkan device, with the first
band taking the remainder (src/ray_trace.cpp:74-93), and never moves pixels between GPUs (each
device presents its own window, :96-105). Here, one process per GPU (torch.distributed over
RCCL): rank r renders the 8-row strips k with k % world == r — interleaving balances sky-heavy
and sphere-heavy rows without the reference's tuner (src/workload_tuner.hpp) — and one gather
per buffer brings every rank's strips to rank 0, where rt_scatter_rows puts them in place.

Pixels are independent and seeds are global (RT_SEED_GLOBAL), so the assembled image is
bit-identical to a one-GPU render whatever the world size.

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
    gathered band into the full image.
    """

    def __init__(self, width: int, height: int, device, render_band: Callable,
                 assemble: Optional[Callable] = None, strip: int = STRIP, gather_accum: bool = True):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.W, self.H, self.device = width, height, device
        self.render_band = render_band
        self.assemble = assemble
        self.gather_accum = gather_accum
        self.rows_np = strip_rows(self.rank, self.world, height, strip)
        self.nmax = max_rows(self.world, height, strip)
        n = len(self.rows_np)
        # Bands are padded to the largest band so one fixed-size gather moves every rank's rows.
        # one rank: the identity map is left out (no per-sample row lookup in the kernel)
        self.rows = torch.from_numpy(self.rows_np).to(device) if self.world > 1 else None
        self.accum = torch.zeros((self.nmax, width, 4), dtype=torch.float32, device=device)
        self.out = torch.zeros((self.nmax, width, 4), dtype=torch.uint8, device=device)
        self.n = n
        # gloo moves host tensors only: stage device bands through host memory (rehearsal of the
        # multi-rank path on a shared GPU; RCCL gathers device memory directly).
        self.staged = (self.world > 1 and getattr(device, "type", str(device)) != "cpu"
                       and dist.get_backend() == "gloo")
        if self.rank == 0:
            self.all_rows = [torch.from_numpy(strip_rows(r, self.world, height, strip)).to(device)
                             for r in range(self.world)]
            self.g_accum = [torch.empty_like(self.accum) for _ in range(self.world)]
            self.g_out = [torch.empty_like(self.out) for _ in range(self.world)]
            self.full_accum = torch.zeros((height, width, 4), dtype=torch.float32, device=device)
            self.full_out = torch.zeros((height, width, 4), dtype=torch.uint8, device=device)

    def step(self):
        """Render this rank's strips, gather to rank 0, assemble. Returns (accum, rgba8) of the
        full image on rank 0, None elsewhere."""
        self.render_band(self.rows, self.accum[: self.n], self.out[: self.n])
        if self.world == 1:
            return self.accum[: self.n], self.out[: self.n]
        if self.gather_accum:
            self._gather(self.accum, self.g_accum if self.rank == 0 else None)
        self._gather(self.out, self.g_out if self.rank == 0 else None)
        if self.rank != 0:
            return None
        for r in range(self.world):
            rows = self.all_rows[r]
            k = rows.numel()
            self.assemble(self.g_accum[r][:k] if self.gather_accum else None, self.g_out[r][:k], rows,
                          self.full_accum if self.gather_accum else None, self.full_out)
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


_force_collective = False   # tests: take the RCCL code path with an emulated all_to_all_single


def split_samples(spp: int, world: int) -> list:
    """spp_r of every rank: as even as possible, sum = spp (ranks beyond spp get 0)."""
    return [spp // world + (1 if r < spp % world else 0) for r in range(world)]


def row_slices(height: int, world: int) -> list:
    """Row counts of the all-to-all reduction slices (contiguous, as even as possible)."""
    return [height // world + (1 if r < height % world else 0) for r in range(world)]


class SampleSplitRenderer:
    """One rank's share of a sample-split multi-GPU frame (module docstring).

    render_full(number, spp_r, accum_dev, out_dev): renders the whole frame with spp_r samples and
    stream salt `number` into [H, W, 4] buffers. reduce(slices, spp, accum_out, out): accum_out =
    float sum of slices[0..N) in order with alpha 1, out = its rgba8 tonemap (rt_reduce_resolve).
    """

    def __init__(self, width: int, height: int, spp: int, number: int, device, render_full: Callable,
                 reduce: Callable):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.W, self.H, self.spp, self.device = width, height, spp, device
        self.spp_r = split_samples(spp, self.world)[self.rank]
        self.number = number + self.rank
        self.render_full, self.reduce = render_full, reduce
        self.accum = torch.zeros((height, width, 4), dtype=torch.float32, device=device)
        self.out = torch.zeros((height, width, 4), dtype=torch.uint8, device=device)
        self.rows = row_slices(height, self.world)
        self.row0 = [sum(self.rows[:r]) for r in range(self.world)]
        self.n_max = max(self.rows)
        n_mine = self.rows[self.rank]
        # received slices, rank-major: the collective sees [N * rows, W, 4], the reduction [N, rows, W, 4]
        self.recv_flat = torch.empty((self.world * n_mine, width, 4), dtype=torch.float32, device=device)
        self.recv = self.recv_flat.view(self.world, n_mine, width, 4)
        # reduced slice, padded to n_max rows so every rank's gather buffer has one shape
        self.part = torch.zeros((self.n_max, width, 4), dtype=torch.float32, device=device)
        self.part_out = torch.zeros((self.n_max, width, 4), dtype=torch.uint8, device=device)
        # gloo has no all_to_all: host staging + one scatter per root (rehearsal / CPU tests)
        self.gloo = self.world > 1 and dist.get_backend() == "gloo" and not _force_collective
        self.even = all(n == self.n_max for n in self.rows)
        self.multi = self.world > 1 or _force_collective   # exchange even at N = 1 (tests)
        if self.rank == 0 and self.multi:
            self.g_accum = torch.zeros((self.world, self.n_max, width, 4), dtype=torch.float32, device=device)
            self.g_out = torch.zeros((self.world, self.n_max, width, 4), dtype=torch.uint8, device=device)
            if self.even:   # the gather lands in place
                self.full_accum = self.g_accum.view(height, width, 4)
                self.full_out = self.g_out.view(height, width, 4)
            else:
                self.full_accum = torch.zeros((height, width, 4), dtype=torch.float32, device=device)
                self.full_out = torch.zeros((height, width, 4), dtype=torch.uint8, device=device)

    def step(self):
        """Render this rank's samples, reduce, tonemap, gather. Returns (accum, rgba8) of the whole
        frame on rank 0, None elsewhere."""
        torch, dist = self.torch, self.dist
        if not self.multi:
            self.render_full(self.number, self.spp_r, self.accum, self.out)
            return self.accum, self.out
        if self.spp_r:
            self.render_full(self.number, self.spp_r, self.accum, self.out)
        else:
            self.accum.zero_()
        W, r, n_mine = self.W, self.rank, self.rows[self.rank]
        # all-to-all: rank q receives row slice q of every rank's accumulator, in rank order
        if self.gloo:   # rehearsal backend (no all_to_all): host staging, scatter from every root
            hs = []
            for q in range(self.world):
                h = torch.zeros((self.n_max, W, 4), dtype=torch.float32)
                h[: self.rows[q]].copy_(self.accum[self.row0[q]: self.row0[q] + self.rows[q]])
                hs.append(h)
            hr = torch.empty((self.n_max, W, 4), dtype=torch.float32)
            for q in range(self.world):
                dist.scatter(hr, hs if q == r else None, src=q)
                self.recv[q].copy_(hr[:n_mine])
        else:
            dist.all_to_all_single(self.recv_flat, self.accum, output_split_sizes=[n_mine] * self.world,
                                   input_split_sizes=self.rows)
        self.reduce(self.recv, self.spp, self.part[:n_mine], self.part_out[:n_mine])
        self._gather(self.part, self.g_accum if r == 0 else None)
        self._gather(self.part_out, self.g_out if r == 0 else None)
        if r != 0:
            return None
        if not self.even:
            for q in range(self.world):
                self.full_accum[self.row0[q]: self.row0[q] + self.rows[q]].copy_(self.g_accum[q, : self.rows[q]])
                self.full_out[self.row0[q]: self.row0[q] + self.rows[q]].copy_(self.g_out[q, : self.rows[q]])
        return self.full_accum, self.full_out

    def _gather(self, t, dst):
        """Gather every rank's [n_max, W, 4] slice into dst[world, n_max, W, 4] on rank 0."""
        dist = self.dist
        lst = list(dst.unbind(0)) if dst is not None else None
        if self.gloo:
            hb = t.cpu()
            hl = [self.torch.empty_like(hb) for _ in range(self.world)] if lst is not None else None
            dist.gather(hb, hl, dst=0)
            if lst is not None:
                for d, h in zip(lst, hl):
                    d.copy_(h)
        else:
            dist.gather(t, lst, dst=0)


def hip_full_renderer(renderer, rci, options, stream=None):
    """render_full backed by librt_mi355x.so: the whole frame with spp_r samples, salt `number`."""
    import copy

    def render_full(number, spp_r, accum, out):
        rc = copy.copy(rci)
        rc.number = number
        rc.samplesPerRenderCall = spp_r
        renderer.render_device(rc, accum, out, options=options, stream=stream)
    return render_full


def hip_reducer(renderer, stream=None):
    """reduce backed by rt_reduce_resolve (one pass: rank-ordered sum + tonemap)."""
    def reduce(slices, spp, accum_out, out):
        renderer.reduce_resolve(slices, spp, accum_out, out, stream=stream)
    return reduce
