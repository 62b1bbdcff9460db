"""GPU parity: librt_mi355x.so (through its C-ABI) against the CPU oracle on the same inputs.

Bar: bit-exact. Both sides implement the arithmetic contract of DESIGN.md §3 (IEEE binary32,
explicit fmas, correctly rounded divide/sqrt, deterministic sin), so every accumulator float and
every rgba8 byte must be identical, and the traced-segment counts must agree. Full-size cases
use size-independent properties (LBVH == brute force, band-split invariance) plus one full-frame
oracle comparison at 1 spp.
"""
import contextlib
import ctypes
import json
import os
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"
BRUTE, LBVH = 1, 2
LBVH_ORDERED = 3   # test-only alias: accel LBVH with the ordered two-wide walk (options.reserved[1] = 2)
LBVH_COMPACT = 4   # test-only alias: accel LBVH, escape-link walk over 16-B nodes (options.reserved[1] = 4)
LBVH_POOL = 5      # test-only alias: accel LBVH, LDS scene + tail-compaction pool (options.reserved[1] = 7)
LBVH_OCT = 6       # test-only alias: accel LBVH, octant-specialised node copies in LDS (options.reserved[1] = 8)
WALK_FORM = {LBVH_ORDERED: 2, LBVH_COMPACT: 4, LBVH_POOL: 7, LBVH_OCT: 8}
HOST_TREE_FORMS = (LBVH_ORDERED, LBVH_COMPACT)


@contextlib.contextmanager
def tree_builder(kind):
    """RT_BVH_BUILD (gpu | sah | morton) for the scenes set inside; the walk A/B forms need a
    host-built tree."""
    prev = os.environ.get("RT_BVH_BUILD")
    if kind:
        os.environ["RT_BVH_BUILD"] = kind
    try:
        yield
    finally:
        if prev is None:
            os.environ.pop("RT_BVH_BUILD", None)
        else:
            os.environ["RT_BVH_BUILD"] = prev


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def rtvk(torch):
    import rtvk as m
    return m


@pytest.fixture(scope="module")
def renderer(rtvk):
    r = rtvk.Renderer(0)
    yield r
    r.close()


def gpu_render(rtvk, renderer, torch, spheres, rci_u32, band_w, band_h, rows=None, accel=LBVH,
               max_depth=50, seed_mode=0, rng_mode=0, accumulate=False, sample_base=0, accum=None,
               count=False, builder=None):
    with tree_builder(builder or ("sah" if accel in HOST_TREE_FORMS else None)):
        renderer.set_scene(np.ascontiguousarray(spheres, np.uint8).reshape(-1, 80))
    rci = rtvk.RenderCallInfo.from_buffer_copy(np.ascontiguousarray(rci_u32).tobytes())
    acc = (torch.zeros((band_h, band_w, 4), dtype=torch.float32, device="cuda") if accum is None
           else torch.from_numpy(np.ascontiguousarray(accum, np.float32)).cuda())
    out = torch.full((band_h, band_w, 4), 7, dtype=torch.uint8, device="cuda")
    rows_t = None if rows is None else torch.from_numpy(np.asarray(rows, np.int32)).cuda()
    opt = rtvk.make_options(max_depth=max_depth, seed_mode=seed_mode, rng_mode=rng_mode,
                            accel=LBVH if accel in WALK_FORM else accel,
                            accumulate=accumulate, sample_base=sample_base, count_tests=count)
    opt.reserved[1] = WALK_FORM.get(accel, 0)
    renderer.render_device(rci, acc, out, rows=rows_t, options=opt)
    torch.cuda.synchronize()
    st = renderer.stats()
    return acc.cpu().numpy(), out.cpu().numpy(), st


def assert_same(a_gpu, o_gpu, a_ref, o_ref):
    diff = np.argwhere(a_gpu != a_ref)
    assert diff.size == 0, f"{len(diff)} accumulator floats differ, first at {diff[:4].tolist()}"
    np.testing.assert_array_equal(o_gpu, o_ref)


# ---- primitives -------------------------------------------------------------------------------
@pytest.mark.parametrize("op", [0, 1, 2, 3, 4, 5])
def test_math_primitives_bit_exact(rtvk, torch, oracle, op):
    rng = np.random.default_rng(op)
    n = 20000
    if op == 0:
        x = np.abs(rng.standard_normal(n)).astype(np.float32) * np.float32(10) ** rng.integers(-20, 20, n).astype(np.float32)
        y = np.zeros(n, np.float32)
        ref = np.sqrt(x)
    elif op == 1:
        x = rng.standard_normal(n).astype(np.float32) * 1e3
        y = rng.standard_normal(n).astype(np.float32)
        ref = x / y
    elif op == 2:
        x = np.concatenate([rng.uniform(-100, 100, n // 2), rng.uniform(-6e4, 6e4, n // 2)]).astype(np.float32)
        y = np.zeros(n, np.float32)
        ref = np.array([oracle.sinf(float(v)) for v in x], np.float32)
    elif op == 3:
        x = rng.standard_normal(n).astype(np.float32)
        y = rng.standard_normal(n).astype(np.float32)
        ref = (x.astype(np.float64) * y.astype(np.float64) + 1.0).astype(np.float32)  # exact fma for f32
    elif op == 4:  # normalize(v) = v * (1 / sqrt(fma(z,z, fma(y,y, x*x)))), v = (x, y, 0.5)
        x = rng.standard_normal(n).astype(np.float32)
        y = rng.standard_normal(n).astype(np.float32)
        xx = x * x
        d = (y.astype(np.float64) * y + xx).astype(np.float32)   # fma: exact product, one rounding
        d = (np.float64(0.25) + d).astype(np.float32)             # fma(0.5, 0.5, d)
        inv = np.float32(1) / np.sqrt(d)
        ref = x * inv
    else:
        x = rng.uniform(-0.5, 1.5, n).astype(np.float32)
        y = np.zeros(n, np.float32)
        x2 = x * x
        ref = np.where(x < 0, np.float32(np.nan), x2 * x2 * x).astype(np.float32)
    pairs = np.ascontiguousarray(np.stack([x, y], 1), np.float32)
    out = np.zeros(n, np.float32)
    from rtvk import abi
    abi.check(rtvk.load_library().rt_debug_math(0, op, pairs.ctypes.data, out.ctypes.data, n))
    same = (out.view(np.uint32) == ref.astype(np.float32).view(np.uint32)) | (np.isnan(out) & np.isnan(ref))
    assert same.all(), f"op {op}: {np.count_nonzero(~same)} differ, e.g. x={x[~same][:3]} gpu={out[~same][:3]} ref={ref[~same][:3]}"


# ---- golden fixtures --------------------------------------------------------------------------
@pytest.mark.parametrize("accel", [BRUTE, LBVH, LBVH_ORDERED, LBVH_COMPACT, LBVH_POOL, LBVH_OCT])
@pytest.mark.parametrize("case", ["g64x36_spp4", "g48x32_spp3_depth3_local", "g40x24_spp2_counter"])
def test_golden(rtvk, renderer, torch, oracle, case, accel):
    m = json.loads((GOLDEN / f"{case}.json").read_text())
    g = np.load(GOLDEN / f"{case}.npz", allow_pickle=False)
    sc = oracle.generate_scene(m["t"], m["K"])
    rci = oracle.render_call_info(m["spp"], m["W"], m["H"], tuple(m["offset"]))
    a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, m["band_w"], m["band_h"], accel=accel,
                          max_depth=m["max_depth"], seed_mode=m["seed_mode"], rng_mode=m["rng_mode"])
    assert_same(a, o, g["accum"], g["rgba8"])
    assert st.segments == int(g["stats"][0]) and st.samples == int(g["stats"][1])


# ---- oracle at the same seed ------------------------------------------------------------------
CASES = [
    # (W, H, offset_y, band_h, spp, t, K, kwargs)
    (96, 54, 0, 54, 6, 0.0, 11, {}),
    (13, 7, 0, 7, 5, 0.0, 11, {}),            # ragged tiles
    (1, 1, 0, 1, 9, 0.0, 11, {}),             # single pixel
    (70, 40, 17, 9, 3, 0.9, 11, {}),          # band with offset, moving spheres
    (64, 36, 0, 36, 4, 0.0, 3, {}),           # small grid
    (50, 30, 0, 30, 3, 0.0, 11, {"max_depth": 2}),
    (50, 30, 5, 20, 3, 0.0, 11, {"seed_mode": 1}),
]


@pytest.mark.parametrize("accel", [BRUTE, LBVH, LBVH_ORDERED, LBVH_COMPACT, LBVH_POOL, LBVH_OCT])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_vs_oracle(rtvk, renderer, torch, oracle, case, accel):
    W, H, oy, bh, spp, t, K, kw = CASES[case]
    sc = oracle.generate_scene(t, K)
    rci = oracle.render_call_info(spp, W, H, (0, oy))
    ra, ro, rst = oracle.render(sc, rci, W, bh, opts=oracle.options(**kw))
    a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, bh, accel=accel, **kw)
    assert_same(a, o, ra, ro)
    assert (st.segments, st.samples) == rst[:2]


def test_empty_and_single_sphere(rtvk, renderer, torch, oracle):
    rci = oracle.render_call_info(2, 20, 10)
    for sc in (np.zeros((0, 80), np.uint8), oracle.generate_scene()[:1], oracle.generate_scene()[3:4]):
        ra, ro, _ = oracle.render(sc, rci, 20, 10)
        for accel in (BRUTE, LBVH, LBVH_ORDERED, LBVH_COMPACT, LBVH_POOL, LBVH_OCT):
            a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, 20, 10, accel=accel)
            assert_same(a, o, ra, ro)


def test_rows_strip_map(rtvk, renderer, torch, oracle):
    W, H = 40, 30
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(3, W, H)
    fa, fo, _ = oracle.render(sc, rci, W, H)
    rows = np.array([29, 0, 8, 9, 10, 15], np.int32)
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, len(rows), rows=rows)
    assert_same(a, o, fa[rows], fo[rows])


def test_accumulate_and_counter_rng(rtvk, renderer, torch, oracle):
    W, H = 24, 16
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(2, W, H)
    base, _, _ = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=1))
    ra, ro, _ = oracle.render(sc, rci, W, H, accum=base, opts=oracle.options(rng_mode=1, accumulate=1, sample_base=2))
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accum=base, rng_mode=1, accumulate=True, sample_base=2)
    assert_same(a, o, ra, ro)


def test_host_rt_render_bands(rtvk, oracle):
    """rt_render with 3 bands (one per GPU in the reference; here all on the visible devices)."""
    W, H = 32, 20
    sc = oracle.generate_scene()
    rcis = [rtvk.canonical_render_call_info(2, W, H) for _ in range(3)]
    for r, y in zip(rcis, (0, 7, 13)):
        r.offset.y = y
    res = rtvk.render(rtvk.generateRandomScene(), rcis)
    ra, ro, _ = oracle.render(sc, oracle.render_call_info(2, W, H), W, H)
    assert_same(res.accum, res.rgba8, ra, ro)


# ---- full size --------------------------------------------------------------------------------
def test_full_frame_1spp_vs_oracle(rtvk, renderer, torch, oracle):
    """Config 1 frame (1920x1080, 1 spp) against the oracle: bit-exact => PSNR = inf >= 50 dB."""
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(1, 1920, 1080)
    ra, ro, rst = oracle.render(sc, rci, 1920, 1080, threads=16)
    a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, 1920, 1080, accel=LBVH)
    n_diff = int(np.count_nonzero(np.any(a != ra, axis=-1)))
    mse = np.mean((o[..., :3].astype(np.float64) - ro[..., :3]) ** 2)
    psnr = float("inf") if mse == 0 else 10 * np.log10(255 ** 2 / mse)
    assert psnr >= 50.0
    assert n_diff == 0, f"{n_diff} pixels differ (PSNR {psnr:.1f} dB)"
    assert (st.segments, st.samples) == rst[:2]


@pytest.mark.parametrize("W,H,spp,K", [(1920, 1080, 2, 11), (3840, 2160, 1, 11), (256, 144, 1, 158)])
def test_lbvh_equals_brute_full_size(rtvk, renderer, torch, oracle, W, H, spp, K):
    sc = oracle.generate_scene(0.0, K)
    rci = oracle.render_call_info(spp, W, H)
    ab, ob, sb = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=BRUTE)
    for builder in ("gpu", "sah", "morton"):
        al, ol, sl = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH, builder=builder)
        assert_same(al, ol, ab, ob)
        assert sb.segments == sl.segments
    for form in (LBVH_ORDERED, LBVH_COMPACT, LBVH_POOL, LBVH_OCT):
        ao, oo, so = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=form)
        assert_same(ao, oo, ab, ob)


def test_band_split_invariance_full_size(rtvk, renderer, torch, oracle):
    sc = oracle.generate_scene()
    W, H = 1920, 1080
    rci = oracle.render_call_info(1, W, H)
    fa, fo, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H)
    rows = np.arange(H, dtype=np.int32).reshape(-1, 8)[1::3].reshape(-1)   # every third 8-row strip
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, len(rows), rows=rows)
    assert_same(a, o, fa[rows], fo[rows])


def test_lpt_schedule_same_image(rtvk, renderer, torch, oracle):
    """The second launch over a band geometry hands tiles out longest pixel chain first (the
    first launch's costs): every tile's key is a real chain length (spp .. spp x depth
    segments), and the image and the counts are unchanged and equal the oracle."""
    sc = oracle.generate_scene()
    W, H, spp = 100, 60, 3   # ragged 8x8 tiles
    rci = oracle.render_call_info(spp, W, H)
    ra, ro, rst = oracle.render(sc, rci, W, H)
    a0, o0, s0 = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH)
    cost = renderer.tile_costs()
    assert cost.shape == (((W + 7) // 8) * ((H + 7) // 8),)
    assert (cost >= spp).all() and (cost <= spp * 50).all() and len(np.unique(cost)) > 4
    a1, o1, s1 = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH)
    assert_same(a0, o0, ra, ro)
    assert_same(a1, o1, ra, ro)
    assert (s1.segments, s1.samples) == (s0.segments, s0.samples) == rst[:2]
    np.testing.assert_array_equal(renderer.tile_costs(), cost)


def test_count_variant_same_image(rtvk, renderer, torch, oracle):
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(2, 128, 72)
    a0, o0, s0 = gpu_render(rtvk, renderer, torch, sc, rci, 128, 72, accel=LBVH)
    a1, o1, s1 = gpu_render(rtvk, renderer, torch, sc, rci, 128, 72, accel=LBVH, count=True)
    assert_same(a1, o1, a0, o0)
    assert s1.box_tests > 0 and s1.sphere_tests > 0 and s0.box_tests == 0


@pytest.mark.parametrize("cam", [(500.0, 300.0, -200.0), (0.0, 4000.0, 0.5), (13.0, 0.05, -3.0)])
def test_far_and_grazing_cameras(rtvk, renderer, torch, oracle, cam):
    """Cameras outside the padded scene radius force a re-pad of the LBVH boxes; a camera just
    above the ground makes grazing primary rays. LBVH must equal brute force and the oracle."""
    W, H = 48, 32
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(2, W, H)
    f = rci.view(np.float32)
    f[8:11] = cam
    f[12:15] = [-cam[0], -cam[1], -cam[2]]
    ra, ro, _ = oracle.render(sc, rci, W, H)
    for accel in (BRUTE, LBVH, LBVH_ORDERED, LBVH_COMPACT):
        a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel)
        assert_same(a, o, ra, ro)
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH, builder="gpu")
    assert_same(a, o, ra, ro)


def test_scatter_rows_reassembles_strips(rtvk, renderer, torch, oracle):
    """The multi-GPU reassembly on device: strips rendered through row maps, scattered back with
    rt_scatter_rows, equal the full-frame render (rtvk.dist's rank-0 step)."""
    from rtvk.dist import strip_rows
    W, H, world = 64, 45, 3
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(2, W, H)
    ra, ro, _ = oracle.render(sc, rci, W, H)
    renderer.set_scene(sc)
    rci_c = rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes())
    full_a = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    full_o = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    for rank in range(world):
        rows = torch.from_numpy(strip_rows(rank, world, H)).cuda()
        a = torch.zeros((rows.numel(), W, 4), dtype=torch.float32, device="cuda")
        o = torch.zeros((rows.numel(), W, 4), dtype=torch.uint8, device="cuda")
        renderer.render_device(rci_c, a, o, rows=rows, options=rtvk.make_options())
        renderer.scatter_rows(a, o, rows, full_a, full_o)
    torch.cuda.synchronize()
    assert_same(full_a.cpu().numpy(), full_o.cpu().numpy(), ra, ro)


@pytest.mark.parametrize("form", [LBVH, LBVH_OCT, LBVH_POOL])
def test_lbvh_equals_brute_bench_workload(rtvk, renderer, torch, oracle, form):
    """The bench frame itself (1920x1080, 100 spp, canonical scene): ~5.9e8 traced segments, so
    rare rays (a direction component that is exactly zero, grazing hits) all occur; every
    accumulator float and rgba8 byte of the LBVH walk equals brute force."""
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(100, 1920, 1080)
    ab, ob, sb = gpu_render(rtvk, renderer, torch, sc, rci, 1920, 1080, accel=BRUTE)
    al, ol, sl = gpu_render(rtvk, renderer, torch, sc, rci, 1920, 1080, accel=form)
    bad = np.argwhere(np.any(al != ab, axis=-1))
    assert bad.size == 0, f"{len(bad)} pixels differ from brute force, first {bad[:4].tolist()}"
    np.testing.assert_array_equal(ol, ob)
    assert (sl.segments, sl.samples) == (sb.segments, sb.samples)


def test_resolve_rgba8_edge_values(rtvk, renderer, torch, oracle):
    """rt_resolve_rgba8 against the oracle's tonemap on edge accumulators: negative, zero,
    subnormal, > spp, inf and NaN sums (UNORM clamp, NaN -> 0)."""
    rng = np.random.default_rng(5)
    a = rng.standard_normal((37, 53, 4)).astype(np.float32) * 40
    special = np.array([0.0, -0.0, 1e-45, -1e-45, np.inf, -np.inf, np.nan, 99.5, 100.0, 1e30], np.float32)
    a.reshape(-1)[: special.size * 7] = np.tile(special, 7)
    for spp in (1, 3, 100):
        out = torch.zeros((37, 53, 4), dtype=torch.uint8, device="cuda")
        renderer.resolve_rgba8(torch.from_numpy(a).cuda(), spp, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), oracle.resolve(a, spp))
    with pytest.raises(rtvk.RtError):
        renderer.resolve_rgba8(torch.from_numpy(a).cuda(), 0, out)


@pytest.mark.parametrize("world", [2, 3])
def test_sample_split_subframes(rtvk, renderer, torch, oracle, world):
    """The sample-split multi-GPU frame (rtvk.dist.SampleSplitRenderer) on one device: the sub-frame
    of each simulated rank (spp_r samples, number = 7 + r) equals the oracle's, and
    rt_reduce_resolve of the stacked sub-frames equals their float sum in rank order (alpha 1)
    and its tonemap, bit for bit."""
    from rtvk.dist import split_samples
    W, H, spp = 72, 40, 5
    sc = oracle.generate_scene()
    renderer.set_scene(sc)
    slices = torch.zeros((world, H, W, 4), dtype=torch.float32, device="cuda")
    ref = None
    for r, s in enumerate(split_samples(spp, world)):
        rci = oracle.render_call_info(s, W, H, number=7 + r)
        o = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        renderer.render_device(rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes()), slices[r], o,
                               options=rtvk.make_options())
        ra, ro, _ = oracle.render(sc, rci, W, H)
        torch.cuda.synchronize()
        assert_same(slices[r].cpu().numpy(), o.cpu().numpy(), ra, ro)
        ref = ra if ref is None else ref + ra
    ref[..., 3] = 1.0
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    renderer.reduce_resolve(slices, spp, acc, out)
    torch.cuda.synchronize()
    assert_same(acc.cpu().numpy(), out.cpu().numpy(), ref, oracle.resolve(ref, spp))
    # in place over slice 0 (the accum_out alias the library allows)
    renderer.reduce_resolve(slices, spp, slices[0], out)
    torch.cuda.synchronize()
    assert_same(slices[0].cpu().numpy(), out.cpu().numpy(), ref, oracle.resolve(ref, spp))


@pytest.mark.parametrize("reserve", ["0", "100", str(1 << 40)])
def test_chunked_refill_same_image(rtvk, renderer, torch, oracle, reserve):
    """Pixel hand-out by whole tiles (RT_REFILL_RESERVE=0), tiles then single pixels (100), and
    single pixels only (huge reserve) render the same image as the oracle, on a ragged frame
    (width and height not multiples of 8) so tiles with missing pixels go through the tile path."""
    W, H = 203, 117
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(3, W, H)
    ra, ro, rs = oracle.render(sc, rci, W, H)
    prev = os.environ.get("RT_REFILL_RESERVE")
    os.environ["RT_REFILL_RESERVE"] = reserve
    try:
        for _ in range(2):   # second launch runs with the LPT hand-out order
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH_OCT)
            assert_same(a, o, ra, ro)
            assert (st.segments, st.samples) == (rs[0], rs[1])
    finally:
        if prev is None:
            os.environ.pop("RT_REFILL_RESERVE", None)
        else:
            os.environ["RT_REFILL_RESERVE"] = prev


def test_scene_swap_between_queued_frames(rtvk, renderer, torch, oracle):
    """rt_set_scene does not wait for queued frames: a frame queued before the call renders the
    old scene, one queued after renders the new one (upload in stream order), over four frames
    so both pinned staging buffers are reused."""
    W, H, spp = 96, 64, 2
    scenes = [oracle.generate_scene(t) for t in (0.0, 1.0, 2.0, 0.5)]
    rci = oracle.render_call_info(spp, W, H)
    rci_c = rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes())
    accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in scenes]
    outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in scenes]
    torch.cuda.synchronize()
    for sc, a, o in zip(scenes, accs, outs):
        renderer.set_scene(sc)
        renderer.render_device(rci_c, a, o, options=rtvk.make_options())
    torch.cuda.synchronize()
    for sc, a, o in zip(scenes, accs, outs):
        ra, ro, _ = oracle.render(sc, rci, W, H)
        assert_same(a.cpu().numpy(), o.cpu().numpy(), ra, ro)


def test_sample_split_rccl_world1(rtvk, renderer, torch, oracle):
    """The RCCL code path of rtvk.dist.SampleSplitRenderer (all_to_all_single into the flat receive
    buffer, rt_reduce_resolve, in-place gathers) on a one-rank NCCL group: the frame equals the
    one-GPU render bit for bit."""
    import socket
    import torch.distributed as dist
    import rtvk.dist as rd
    W, H, spp = 80, 48, 3
    sc = oracle.generate_scene()
    renderer.set_scene(sc)
    rci = rtvk.RenderCallInfo.from_buffer_copy(oracle.render_call_info(spp, W, H).tobytes())
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        rd._force_collective = True
        sr = rd.SampleSplitRenderer(W, H, spp, 0, torch.device("cuda", 0),
                                    rd.hip_full_renderer(renderer, rci, rtvk.make_options()),
                                    rd.hip_reducer(renderer))
        acc, out = sr.step()
        torch.cuda.synchronize()
    finally:
        rd._force_collective = False
        dist.destroy_process_group()
    ra, ro, _ = oracle.render(sc, oracle.render_call_info(spp, W, H), W, H)
    assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra, ro)


@pytest.mark.parametrize("isolate", ["0", "3", "1000000"])
def test_isolated_tiles_same_image(rtvk, renderer, torch, oracle, isolate):
    """Waves starting on the longest-chain tiles that take no further pixels (RT_ISOLATE_TILES,
    including every wave isolated) render the same image as the oracle; the second launch has
    the LPT order the isolation needs."""
    W, H = 136, 72
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(2, W, H)
    ra, ro, _ = oracle.render(sc, rci, W, H)
    prev = {k: os.environ.get(k) for k in ("RT_ISOLATE_TILES", "RT_REFILL_RESERVE")}
    os.environ["RT_ISOLATE_TILES"] = isolate
    os.environ["RT_REFILL_RESERVE"] = "0"
    try:
        renderer.set_scene(sc)
        rci_c = rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes())
        for _ in range(2):
            a = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
            o = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
            renderer.render_device(rci_c, a, o, options=rtvk.make_options())
            torch.cuda.synchronize()
            assert_same(a.cpu().numpy(), o.cpu().numpy(), ra, ro)
    finally:
        for k, v in prev.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v



@pytest.mark.parametrize("W,H,spp,K,form", [(320, 180, 2, 158, 0), (320, 180, 2, 158, 10), (96, 64, 3, 40, 0)])
def test_treelet_walk_equals_brute(rtvk, renderer, torch, oracle, W, H, spp, K, form):
    """Trees too big for LDS (device-built): the top levels staged in LDS as a treelet, subtrees
    below the cut from L2 (ACCEL_LBVH_TOP, walk form 0) and the all-L2 walk (form 10) equal brute
    force bit for bit, twice each (the second launch runs with the LPT order)."""
    sc = oracle.generate_scene(0.0, K)
    rci = oracle.render_call_info(spp, W, H)
    ab, ob, sb = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=BRUTE)
    for _ in range(2):
        with tree_builder("gpu"):
            renderer.set_scene(np.ascontiguousarray(sc, np.uint8).reshape(-1, 80))
        rc = rtvk.RenderCallInfo.from_buffer_copy(np.ascontiguousarray(rci).tobytes())
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        opt = rtvk.make_options(accel=LBVH)
        opt.reserved[1] = form
        renderer.render_device(rc, acc, out, options=opt)
        torch.cuda.synchronize()
        assert_same(acc.cpu().numpy(), out.cpu().numpy(), ab, ob)
        st = renderer.stats()
        assert (st.segments, st.samples) == (sb.segments, sb.samples)


def test_treelet_after_refit(rtvk, renderer, torch, oracle):
    """The treelet is rebuilt after a refit of a device-built tree (moving spheres): the treelet
    walk still equals brute force on the refitted scene."""
    W, H, spp, K = 128, 72, 2, 40
    sc0, sc1 = oracle.generate_scene(0.0, K), oracle.generate_scene(0.7, K)
    rci = oracle.render_call_info(spp, W, H)
    ab, ob, _ = gpu_render(rtvk, renderer, torch, sc1, rci, W, H, accel=BRUTE)
    with tree_builder("gpu"):
        renderer.set_scene(np.ascontiguousarray(sc0, np.uint8).reshape(-1, 80))
        rc = rtvk.RenderCallInfo.from_buffer_copy(np.ascontiguousarray(rci).tobytes())
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        renderer.render_device(rc, acc, out, options=rtvk.make_options(accel=LBVH))   # treelet of sc0
        renderer.refit_scene(np.ascontiguousarray(sc1, np.uint8).reshape(-1, 80))
        renderer.render_device(rc, acc, out, options=rtvk.make_options(accel=LBVH))
    torch.cuda.synchronize()
    assert_same(acc.cpu().numpy(), out.cpu().numpy(), ab, ob)


@pytest.mark.parametrize("cam", [(500.0, 300.0, -200.0), (13.0, 0.05, -3.0)])
def test_treelet_far_camera(rtvk, renderer, torch, oracle, cam):
    """A device-built tree too big for LDS under a far camera (re-pad of the node boxes, so the
    treelet is rebuilt) and a grazing one: the treelet walk equals brute force."""
    W, H, K = 64, 40, 40
    sc = oracle.generate_scene(0.0, K)
    rci = oracle.render_call_info(2, W, H)
    f = rci.view(np.float32)
    f[8:11] = cam
    f[12:15] = [-cam[0], -cam[1], -cam[2]]
    ab, ob, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=BRUTE)
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH, builder="gpu")
    assert_same(a, o, ab, ob)


@pytest.mark.parametrize("spp,depth", [(0, 50), (1, 1), (5, 0)])
def test_degenerate_sample_and_depth_counts(rtvk, renderer, torch, oracle, spp, depth):
    """spp = 0 (every pixel stored at once: 0/0 tonemaps to 0, alpha 255), depth 1 (one segment
    per sample: no scattered light) and max_depth 0 (the reference default of 50) match the
    oracle bit for bit, with the same segment/sample counts, on the production (octant) walk
    and on brute force."""
    W, H = 40, 24
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(spp, W, H)
    ra, ro, rs = oracle.render(sc, rci, W, H, opts=oracle.options(max_depth=depth if depth else 50))
    for accel in (BRUTE, LBVH):
        a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, max_depth=depth)
        assert_same(a, o, ra, ro)
        assert (st.segments, st.samples) == (rs[0], rs[1])


def test_band_dimension_limits(rtvk, renderer, torch, oracle):
    """Bands wider or taller than 65535 pixels are refused (the kernel packs band coordinates into
    16-bit halves); an empty band is a no-op."""
    renderer.set_scene(oracle.generate_scene())
    rci = rtvk.RenderCallInfo.from_buffer_copy(oracle.render_call_info(1, 70000, 8).tobytes())
    acc = torch.zeros((1, 70000, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((1, 70000, 4), dtype=torch.uint8, device="cuda")
    with pytest.raises(rtvk.RtError):
        renderer.render_device(rci, acc, out, options=rtvk.make_options())
