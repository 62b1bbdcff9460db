"""Multi-GPU path (rtvk.dist) on CPU: world size 2 over gloo, the oracle rendering each rank's
row strips. Checks the strip partition and that gather + reassembly reproduce the one-device
image bit for bit (global seeds make the image independent of the split)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rtvk.dist import max_rows, strip_rows

W, H, SPP = 40, 27, 2


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("height", [1, 7, 27, 1080])
def test_strip_partition(world, height):
    parts = [strip_rows(r, world, height) for r in range(world)]
    allr = np.concatenate(parts)
    assert sorted(allr.tolist()) == list(range(height))
    sizes = [len(p) for p in parts]
    assert max(sizes) - min(sizes) <= 8 and max(sizes) == max_rows(world, height)
    for p in parts:
        assert np.all(np.diff(p) > 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path, rng_mode=0, resolve_on_root=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    from rtvk.dist import DistributedRenderer

    sc = oracle.generate_scene()
    rci = oracle.render_call_info(SPP, W, H)

    def render_band(rows, accum, out):
        r = rows.numpy().astype(np.uint32)
        if r.size:
            a, o, _ = oracle.render(sc, rci, W, len(r), rows=r, opts=oracle.options(rng_mode=rng_mode), threads=2)
            accum.copy_(torch.from_numpy(a))
            out.copy_(torch.from_numpy(o))

    def assemble(band_accum, band_out, rows, full_accum, full_out):
        full_accum[rows.long()] = band_accum
        if full_out is not None:
            full_out[rows.long()] = band_out

    def resolve(full_accum, full_out):   # rank 0 tonemaps the gathered accumulator once
        full_out.copy_(torch.from_numpy(oracle.resolve(full_accum.numpy(), SPP)))

    dr = DistributedRenderer(W, H, torch.device("cpu"), render_band, assemble,
                             resolve=resolve if resolve_on_root else None)
    assert (dr.g_out is None) == resolve_on_root if rank == 0 else True
    res = dr.step()
    if rank == 0:
        np.savez(out_path, accum=res[0].numpy(), rgba8=res[1].numpy())
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rng_mode,resolve_on_root", [(2, 0, True), (2, 2, True), (3, 2, True), (2, 2, False)])
def test_gather_reassembly(tmp_path, oracle, world, rng_mode, resolve_on_root):
    """Strips on `world` gloo ranks, gathered and reassembled on rank 0, equal the one-device
    frame bit for bit, for the reference stream (rng_mode 0) and the counter-based stream (2):
    accumulators gathered and tonemapped once on rank 0 (the default of the bench path), or both
    images gathered."""
    port = _free_port()
    out = str(tmp_path / "img.npz")
    mp.start_processes(_worker, args=(world, port, out, rng_mode, resolve_on_root), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    ref_a, ref_o, _ = oracle.render(oracle.generate_scene(), oracle.render_call_info(SPP, W, H), W, H,
                                    opts=oracle.options(rng_mode=rng_mode))
    np.testing.assert_array_equal(got["accum"], ref_a)
    np.testing.assert_array_equal(got["rgba8"], ref_o)
