"""Multi-GPU path (rtvk.dist) on CPU: world size 2, 3 and 8 (the driver's N = 8 topology) over
gloo, the oracle rendering each rank's rows. Checks the row-exact strip partition (equal to rt_partition_strips, the C++ rt_multi's),
that gather + reassembly reproduce the one-device image bit for bit (global seeds make the image
independent of the split), and the cross-rank balancer:
every rank re-deals the same partition from a synthetic per-row cost, the image stays exact every
frame, and the imbalance falls."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rtvk.dist import max_rows, strip_rows

W, H, SPP = 40, 27, 2


@pytest.mark.parametrize("world", [1, 2, 3, 7, 8])
@pytest.mark.parametrize("height", [1, 7, 27, 1080, 2160])
def test_strip_partition(world, height):
    """Row-exact: every rank holds floor(H / N) or ceil(H / N) rows (round 5's 8-row strips gave
    rank 7 of 8 128 rows at 1080 and the others 136); identical to the C++ partition."""
    import rtvk
    parts = [strip_rows(r, world, height) for r in range(world)]
    allr = np.concatenate(parts)
    assert sorted(allr.tolist()) == list(range(height))
    sizes = [len(p) for p in parts]
    assert max(sizes) - min(sizes) <= 1 and max(sizes) == max_rows(world, height)
    assert max(sizes) == -(-height // world)
    for p in parts:
        assert np.all(np.diff(p) > 0)
    for a, b in zip(parts, rtvk.partition_strips(world, height)):
        np.testing.assert_array_equal(a, b)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path, rng_mode=0, resolve_on_root=True, gather_accum=True):
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
        if full_accum is not None:
            full_accum[rows.long()] = band_accum
        if full_out is not None:
            full_out[rows.long()] = band_out

    def resolve(full_accum, full_out):   # rank 0 tonemaps the gathered accumulator once
        full_out.copy_(torch.from_numpy(oracle.resolve(full_accum.numpy(), SPP)))

    dr = DistributedRenderer(W, H, torch.device("cpu"), render_band, assemble,
                             resolve=resolve if resolve_on_root else None, gather_accum=gather_accum)
    if rank == 0:   # rgba8 gathered exactly when rank 0 does not resolve (resolve without accumulators)
        assert (dr.g_out is None) == (resolve_on_root and gather_accum)
    res = dr.step()
    if rank == 0:
        np.savez(out_path, accum=res[0].numpy(), rgba8=res[1].numpy())
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rng_mode,resolve_on_root,gather_accum",
                         [(2, 0, True, True), (2, 2, True, True), (3, 2, True, True), (2, 2, False, True),
                          (2, 2, True, False), (8, 2, True, True)])
def test_gather_reassembly(tmp_path, oracle, world, rng_mode, resolve_on_root, gather_accum):
    """Strips on `world` gloo ranks, gathered and reassembled on rank 0, equal the one-device
    frame bit for bit, for the reference stream (rng_mode 0) and the counter-based stream (2):
    accumulators gathered and tonemapped once on rank 0 (the default of the bench path), both
    images gathered, or a resolver given without accumulator gathering (only rgba8 travels)."""
    port = _free_port()
    out = str(tmp_path / "img.npz")
    mp.start_processes(_worker, args=(world, port, out, rng_mode, resolve_on_root, gather_accum), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(out)
    ref_a, ref_o, _ = oracle.render(oracle.generate_scene(), oracle.render_call_info(SPP, W, H), W, H,
                                    opts=oracle.options(rng_mode=rng_mode))
    if gather_accum:
        np.testing.assert_array_equal(got["accum"], ref_a)
    np.testing.assert_array_equal(got["rgba8"], ref_o)


BH = 64   # balancing test height: 8 strips


def _row_cost(y):
    """Synthetic per-row kernel cost: rows near the bottom 3x dearer (a sphere-heavy band)."""
    return 1.0 + 2.0 * (y >= 40)


def _balance_worker(rank, world, port, out_path, frames):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    from rtvk.dist import DistributedRenderer

    sc = oracle.generate_scene()
    rci = oracle.render_call_info(SPP, W, BH)
    launched = []   # the rows of every launch of this rank

    def render_band(rows, accum, out):
        r = rows.numpy().astype(np.uint32)
        if r.size:
            launched.append(r.copy())
            a, o, _ = oracle.render(sc, rci, W, len(r), rows=r, opts=oracle.options(rng_mode=2), threads=2)
            accum.copy_(torch.from_numpy(a))
            out.copy_(torch.from_numpy(o))

    def assemble(band_accum, band_out, rows, full_accum, full_out):
        full_accum[rows.long()] = band_accum

    def resolve(full_accum, full_out):
        full_out.copy_(torch.from_numpy(oracle.resolve(full_accum.numpy(), SPP)))

    def timer(back, band_rows):   # the launch `back` before the last: its synthetic time and weights
        rows = launched[len(launched) - 1 - back]
        assert len(rows) == band_rows
        c = np.array([_row_cost(int(y)) for y in rows])
        return float(c.sum()), c

    dr = DistributedRenderer(W, BH, torch.device("cpu"), render_band, assemble, resolve=resolve, timer=timer)
    imb, rows_seen, images = [], [], []
    for _ in range(frames):
        loads = [sum(_row_cost(int(y)) for y in p) for p in dr.parts]
        imb.append(max(loads) / (sum(loads) / len(loads)))
        rows_seen.append(np.concatenate(dr.parts))
        res = dr.step()
        if rank == 0:
            images.append((res[0].numpy().copy(), res[1].numpy().copy()))
    np.save(out_path + f".rows{rank}.npy", np.stack(rows_seen))
    if rank == 0:
        np.savez(out_path, imb=np.array(imb), accum=np.stack([a for a, _ in images]),
                 rgba8=np.stack([o for _, o in images]), rebalances=dr.rebalances, moved=dr.rows_moved)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_balancer_redeals_rows(tmp_path, oracle, world):
    """Cross-rank balancing (rtvk.dist, rt_partition_rebalance): with a synthetic per-row cost that
    makes the bottom rows 3x dearer, the ranks re-deal band-end rows between frames (every rank the
    same partition: lag-2 feedback, costs summed over gloo), every frame's image equals the
    one-device frame bit for bit, and the imbalance of the last frames is below the first's."""
    port = _free_port()
    out = str(tmp_path / "bal.npz")
    frames = 7
    mp.start_processes(_balance_worker, args=(world, port, out, frames), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    ref_a, ref_o, _ = oracle.render(oracle.generate_scene(), oracle.render_call_info(SPP, W, BH), W, BH,
                                    opts=oracle.options(rng_mode=2))
    for f in range(frames):
        np.testing.assert_array_equal(got["accum"][f], ref_a)
        np.testing.assert_array_equal(got["rgba8"][f], ref_o)
    rows = [np.load(out + f".rows{r}.npy") for r in range(world)]
    for r in range(1, world):
        np.testing.assert_array_equal(rows[r], rows[0])   # every rank holds the same partition
    imb = got["imb"]
    assert int(got["rebalances"]) >= 1 and int(got["moved"]) >= 1
    assert imb[-1] < imb[0] - 0.05, imb
    assert imb[-1] <= 1.0 + 3.0 / (sum(_row_cost(y) for y in range(BH)) / world), imb


def test_blend_outside_unit_interval_refused():
    """DistributedRenderer takes rt_multi's balancer settings: blend in (0, 1] (0 would freeze the
    per-row estimates; rt_debug_multi_tune refuses it too)."""
    from rtvk.dist import DistributedRenderer
    for b in (0.0, -0.5, 1.5):
        with pytest.raises(ValueError):
            DistributedRenderer(8, 8, torch.device("cpu"), lambda *a: None, blend=b)
    DistributedRenderer(8, 8, torch.device("cpu"), lambda *a: None, blend=1.0)
