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


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    from rtvk.dist import DistributedRenderer

    sc = oracle.generate_scene()
    rci = oracle.render_call_info(SPP, W, H)

    def render_band(rows, accum, out):
        r = rows.numpy().astype(np.uint32)
        if r.size:
            a, o, _ = oracle.render(sc, rci, W, len(r), rows=r, threads=2)
            accum.copy_(torch.from_numpy(a))
            out.copy_(torch.from_numpy(o))

    def assemble(band_accum, band_out, rows, full_accum, full_out):
        full_accum[rows.long()] = band_accum
        full_out[rows.long()] = band_out

    dr = DistributedRenderer(W, H, torch.device("cpu"), render_band, assemble)
    res = dr.step()
    if rank == 0:
        np.savez(out_path, accum=res[0].numpy(), rgba8=res[1].numpy())
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


def test_gather_reassembly_world2(tmp_path, oracle):
    port = _free_port()
    out = str(tmp_path / "img.npz")
    mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    ref_a, ref_o, _ = oracle.render(oracle.generate_scene(), oracle.render_call_info(SPP, W, H), W, H)
    np.testing.assert_array_equal(got["accum"], ref_a)
    np.testing.assert_array_equal(got["rgba8"], ref_o)


def test_sample_split_partition():
    from rtvk.dist import row_slices, split_samples
    for spp in (1, 3, 100, 1000):
        for world in (1, 2, 3, 8):
            s = split_samples(spp, world)
            assert sum(s) == spp and max(s) - min(s) <= 1
    for h in (1, 27, 1080):
        for world in (1, 2, 8):
            r = row_slices(h, world)
            assert sum(r) == h and max(r) - min(r) <= 1


SPLIT_SPP = 5


def _emulated_all_to_all_single(output, input, output_split_sizes=None, input_split_sizes=None, **_):
    """torch.distributed.all_to_all_single's dim-0 split semantics, built from gloo scatters (gloo
    has no all_to_all): rank r's input chunk q lands in rank q's output chunk r."""
    world, rank = dist.get_world_size(), dist.get_rank()
    ins = list(torch.split(input, input_split_sizes, dim=0))
    outs = list(torch.split(output, output_split_sizes, dim=0))
    sizes = torch.zeros((world, world), dtype=torch.int64)
    sizes[rank] = torch.tensor(input_split_sizes)
    dist.all_reduce(sizes)
    n_max = int(sizes.max())
    tail = tuple(input.shape[1:])
    for src in range(world):
        buf = torch.zeros((n_max,) + tail, dtype=input.dtype)
        lst = None
        if src == rank:
            lst = []
            for q in range(world):
                t = torch.zeros((n_max,) + tail, dtype=input.dtype)
                t[: ins[q].shape[0]] = ins[q]
                lst.append(t)
        dist.scatter(buf, lst, src=src)
        outs[src].copy_(buf[: int(sizes[src, rank])])


def _split_worker(rank, world, port, out_path, force_collective=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    import rtvk.dist as rd
    from rtvk.dist import SampleSplitRenderer
    if force_collective:   # the RCCL code path (all_to_all_single, in-place gathers)
        rd._force_collective = True
        dist.all_to_all_single = _emulated_all_to_all_single

    sc = oracle.generate_scene()

    def render_full(number, spp_r, accum, out):
        a, o, _ = oracle.render(sc, oracle.render_call_info(spp_r, W, H, number=number), W, H, threads=2)
        accum.copy_(torch.from_numpy(a))
        out.copy_(torch.from_numpy(o))

    def reduce(slices, spp, accum_out, out):
        a = slices[0].numpy().copy()
        for q in range(1, slices.shape[0]):
            a += slices[q].numpy()
        a[..., 3] = 1.0
        accum_out.copy_(torch.from_numpy(a))
        out.copy_(torch.from_numpy(oracle.resolve(a, spp)))

    sr = SampleSplitRenderer(W, H, SPLIT_SPP, 7, torch.device("cpu"), render_full, reduce)
    res = sr.step()
    if rank == 0:
        np.savez(out_path, accum=res[0].numpy(), rgba8=res[1].numpy())
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,force_collective", [(2, False), (3, False), (2, True), (3, True), (4, True)])
def test_sample_split_world(tmp_path, oracle, world, force_collective):
    """Rank r renders split_samples(spp)[r] samples with number = 7 + r; the reduced frame equals
    the rank-ordered float sum of those sub-frames, tonemapped with the full spp."""
    from rtvk.dist import split_samples
    port = _free_port()
    out = str(tmp_path / "img.npz")
    mp.start_processes(_split_worker, args=(world, port, out, force_collective), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    sc = oracle.generate_scene()
    ref = None
    for r, s in enumerate(split_samples(SPLIT_SPP, world)):
        a, _, _ = oracle.render(sc, oracle.render_call_info(s, W, H, number=7 + r), W, H)
        ref = a if ref is None else ref + a
    ref[..., 3] = 1.0
    np.testing.assert_array_equal(got["accum"], ref)
    np.testing.assert_array_equal(got["rgba8"], oracle.resolve(ref, SPLIT_SPP))
    # one rank: exactly the reference frame
    a1, o1, _ = oracle.render(sc, oracle.render_call_info(SPLIT_SPP, W, H, number=7), W, H)
    assert not np.array_equal(got["accum"], a1)  # other ranks' salts do change the noise
