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
LBVH_LDS1 = 6      # test-only alias: accel LBVH, one node copy in LDS (options.reserved[1] = 6)
LBVH_GLOBAL = 10   # test-only alias: accel LBVH, every node from L2 (options.reserved[1] = 10)
LBVH_OCT = 8       # test-only alias: accel LBVH, the tree's 8 octant copies in LDS (host trees) or the
                   # treelet (device trees) (options.reserved[1] = 8)
GRID = 12          # test-only alias: the uniform grid (options.reserved[1] = 12)
GRID_COOP = 14     # test-only alias: the uniform grid in LDS, wave-cooperative walk (options.reserved[1] = 14)
GRID_CQ = 16       # test-only alias: the uniform grid in LDS, wave-wide candidate queue (options.reserved[1] = 16)
WALK_FORM = {LBVH_LDS1: 6, LBVH_GLOBAL: 10, LBVH_OCT: 8, GRID: 12, GRID_COOP: 14, GRID_CQ: 16}
FORMS = [BRUTE, LBVH, LBVH_OCT, LBVH_LDS1, LBVH_GLOBAL, GRID_COOP, GRID_CQ]   # LBVH: the default form (the grid for host scenes)
STREAM, COUNTER, HASH = 0, 1, 2


@contextlib.contextmanager
def tuned(renderer, **kv):
    """Launch-plan parameters of the renderer's context for the block (rt_debug_tune; no setting
    may change an image), restored to the defaults afterwards."""
    renderer.tune(**kv)
    try:
        yield
    finally:
        renderer.tune(**{k: None for k in kv})


@contextlib.contextmanager
def tree_builder(kind):
    """RT_BVH_BUILD (gpu | sah | morton) for the scenes set inside."""
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
               count=False, builder=None, regate=False):
    with tree_builder(builder):
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
    if regate:   # every segment's winner recomputed by the deferred AABB gate's fallback
        opt.reserved[0] |= 2
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
    out = _debug_math(rtvk, op, x, y)
    same = (out.view(np.uint32) == ref.astype(np.float32).view(np.uint32)) | (np.isnan(out) & np.isnan(ref))
    assert same.all(), f"op {op}: {np.count_nonzero(~same)} differ, e.g. x={x[~same][:3]} gpu={out[~same][:3]} ref={ref[~same][:3]}"


def test_cheap_exact_rcp_sqrt_exhaustive(rtvk, torch):
    """The kernels' rcp_cr / sqrt_cr (v_rcp_f32 / v_sqrt_f32 + exact fma corrections) equal the
    correctly rounded 1.0f / x and sqrtf(x) for every one of the 2^32 binary32 inputs, and the
    camera's double-reciprocal division equals x / b for every x in [0, 65536) at eleven sizes b."""
    import ctypes
    from rtvk import abi
    bad = (ctypes.c_uint64 * 3)()
    abi.check(rtvk.load_library().rt_debug_exact_exhaustive(0, bad))
    assert tuple(bad) == (0, 0, 0), f"rcp_cr {bad[0]}, sqrt_cr {bad[1]}, camera division {bad[2]} mismatches"


def _debug_math(rtvk, op, x, y):
    pairs = np.ascontiguousarray(np.stack([x, y], 1), np.float32)
    out = np.zeros(len(x), np.float32)
    from rtvk import abi
    abi.check(rtvk.load_library().rt_debug_math(0, op, pairs.ctypes.data, out.ctypes.data, len(x)))
    return out


def test_checker_decision_bit_exact(rtvk, torch, oracle):
    """The kernel decides the checker (shader.rchit:58-60) from the signs of the three sines; the
    oracle multiplies the full sines. Same decision on 60 000 points: uniform, near the zeros of
    sin(6x) (multiples of pi/6), tiny, signed zeros, far (|x| up to 1e4)."""
    rng = np.random.default_rng(21)
    n = 20000
    x = np.concatenate([rng.uniform(-30, 30, n), (rng.integers(-600, 600, n) * np.pi / 6).astype(np.float32)
                        + rng.normal(0, 1e-6, n), rng.uniform(-1e4, 1e4, n)]).astype(np.float32)
    y = np.concatenate([rng.uniform(-1e-5, 1e-5, n), rng.uniform(-3, 3, n), rng.uniform(-1e4, 1e4, n)]).astype(np.float32)
    x[:6] = [0.0, -0.0, 1e-30, -1e-30, np.pi / 6, 0.0]
    y[:6] = [1.0, 1.0, 0.0, -0.0, 1e-38, -0.0]
    z = (np.float32(0.5) * (x - y)).astype(np.float32)
    got = _debug_math(rtvk, 9, x, y)
    # the oracle's product in binary32, left to right, as rt_oracle.cpp texture_color computes it
    ref = np.array([np.float32(np.float32(oracle.sinf(float(np.float32(6) * a))) * np.float32(oracle.sinf(float(np.float32(6) * b))))
                    * np.float32(oracle.sinf(float(np.float32(6) * c))) for a, b, c in zip(x, y, z)], np.float32)
    np.testing.assert_array_equal(got, (ref > 0).astype(np.float32))


def test_hash_primitives_bit_exact(rtvk, torch, oracle):
    """RT_RNG_SAMPLE_HASH primitives: the sample-seed hash (bit patterns) and the 8.24 fixed-point
    conversion of a colour channel (low / high words), device vs oracle."""
    rng = np.random.default_rng(11)
    ps = rng.integers(0, 2**32, 4000, dtype=np.uint64).astype(np.uint32)
    sm = rng.integers(0, 2**20, 4000, dtype=np.uint64).astype(np.uint32)
    got = _debug_math(rtvk, 6, ps.view(np.float32), sm.view(np.float32)).view(np.uint32)
    ref = np.array([oracle.sample_seed_hash(int(a), int(b)) for a, b in zip(ps, sm)], np.uint32)
    np.testing.assert_array_equal(got, ref)
    c = np.concatenate([rng.uniform(0, 1, 3000), 10.0 ** rng.uniform(-40, 0, 3000),
                        [0.0, 1.0, -1.0, 2.0, np.nan, np.inf, 2.0 ** -24, 2.0 ** -25]]).astype(np.float32)
    lo = _debug_math(rtvk, 7, c, np.zeros_like(c)).view(np.uint32).astype(np.uint64)
    hi = _debug_math(rtvk, 8, c, np.zeros_like(c)).view(np.uint32).astype(np.uint64)
    ref = np.array([oracle.sample_fixed(float(v)) for v in c], np.uint64)
    np.testing.assert_array_equal(lo | (hi << np.uint64(32)), ref)


# ---- golden fixtures --------------------------------------------------------------------------
@pytest.mark.parametrize("accel", FORMS)
@pytest.mark.parametrize("case", ["g64x36_spp4", "g48x32_spp3_depth3_local", "g40x24_spp2_counter", "g56x40_spp7_hash"])
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


@pytest.mark.parametrize("accel", FORMS)
@pytest.mark.parametrize("case", range(len(CASES)))
def test_vs_oracle(rtvk, renderer, torch, oracle, case, accel):
    W, H, oy, bh, spp, t, K, kw = CASES[case]
    _vs_oracle(rtvk, renderer, torch, oracle, W, H, oy, bh, spp, t, K, kw, accel)


@pytest.mark.parametrize("accel", FORMS)
@pytest.mark.parametrize("case", [0, 1, 2, 3, 5, 6])
def test_vs_oracle_hash(rtvk, renderer, torch, oracle, case, accel):
    """The same cases in RT_RNG_SAMPLE_HASH mode: per-sample counter streams, chunked over lanes,
    fixed-point sums, resolve kernel: bit-exact vs the oracle's in-order restatement."""
    W, H, oy, bh, spp, t, K, kw = CASES[case]
    _vs_oracle(rtvk, renderer, torch, oracle, W, H, oy, bh, spp, t, K, dict(kw, rng_mode=HASH), accel)


def _vs_oracle(rtvk, renderer, torch, oracle, W, H, oy, bh, spp, t, K, kw, accel):
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
        rh, oh, _ = oracle.render(sc, rci, 20, 10, opts=oracle.options(rng_mode=HASH))
        for accel in FORMS:
            a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, 20, 10, accel=accel)
            assert_same(a, o, ra, ro)
            a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, 20, 10, accel=accel, rng_mode=HASH)
            assert_same(a, o, rh, oh)


@pytest.mark.parametrize("builder", [None, "gpu"])
def test_grid_near_cull_slack_mixed_radii(rtvk, renderer, torch, oracle, builder):
    """The grid walks' small cull slack depends on the smallest and largest small
    radius: a scene of 300 spheres with radii 0.06-0.45 (the grid's 8:1 limit), cameras inside and
    far outside it. The default slack, the full slack (tuning grid_full_slack = 1) and the oracle agree
    bit for bit, both streams, host (LDS) and device (L2) grids."""
    rng = np.random.default_rng(7)
    base = oracle.generate_scene()[4:5]
    recs = [oracle.generate_scene()[:1].copy()]   # the ground sphere
    for _ in range(300):
        r = base.copy()
        rad = float(rng.uniform(0.06, 0.45))
        r[0, :16].view(np.float32)[:] = [rng.uniform(-6, 6), rad, rng.uniform(-6, 6), rad]
        recs.append(r)
    sc = np.concatenate(recs)
    W, H = 48, 32
    for cam, look in [((2.0, 0.6, -3.0), (0.0, 0.3, 0.0)), ((25.0, 9.0, -25.0), (0.0, 0.0, 0.0))]:
        rci = oracle.render_call_info(3, W, H)
        f = rci.view(np.float32)
        f[8:11] = cam
        f[12:15] = [look[k] - cam[k] for k in range(3)]
        for rng_mode in (STREAM, HASH):
            ra, ro, _ = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=rng_mode))
            for full in (None, "1"):
                for accel in (LBVH, GRID_COOP, GRID_CQ):
                    with tuned(renderer, grid_full_slack=full):
                        a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, rng_mode=rng_mode,
                                             builder=builder)
                    assert_same(a, o, ra, ro)


@pytest.mark.parametrize("builder", [None, "gpu"])
def test_grid_lattice_axis_rays(rtvk, renderer, torch, oracle, builder):
    """Uniform-grid stress: spheres on an integer lattice (centers, AABB faces and cell boundaries
    coincide or nearly so), camera looking exactly along +z through the lattice (zero direction
    components, DDA ties at every step) and from a diagonal. Every walk equals brute force and the
    oracle bit for bit; host grid (LDS) and device grid (L2)."""
    sc = oracle.generate_scene()[:1].copy()   # the ground sphere
    recs = [sc]
    base = oracle.generate_scene()[4:5]
    for i in range(-6, 7):
        for j in range(-6, 7):
            r = base.copy()
            g = r[0, :16].view(np.float32)
            g[:] = [float(i), 0.25, float(j), 0.25 if (i + j) % 3 else 0.5]
            recs.append(r)
    sc = np.concatenate(recs)
    W, H = 40, 24
    for cam, look in [((0.0, 0.25, -30.0), (0.0, 0.25, 0.0)), ((9.0, 3.0, -9.0), (0.0, 0.0, 0.0))]:
        rci = oracle.render_call_info(2, W, H)
        f = rci.view(np.float32)
        f[8:11] = cam
        f[12:15] = [look[k] - cam[k] for k in range(3)]
        ra, ro, _ = oracle.render(sc, rci, W, H)
        for accel in (BRUTE, LBVH, GRID, GRID_COOP, GRID_CQ, LBVH_OCT, LBVH_GLOBAL):
            a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, builder=builder)
            assert_same(a, o, ra, ro)


@pytest.mark.parametrize("builder", [None, "gpu"])
def test_more_than_four_big_spheres(rtvk, renderer, torch, oracle, builder):
    """The production kernels test the first four big spheres as one group; a scene with more (the
    canonical scene plus three more radius-1 spheres and one of radius 2.5) takes the general form,
    which loops over the further groups. Grid, tree and brute-force walks equal the oracle bit for
    bit, both streams."""
    sc = oracle.generate_scene()
    extra = []
    for k, (x, z, rad) in enumerate([(0.0, 4.0, 1.0), (-4.0, 4.0, 1.0), (4.0, -4.0, 1.0), (-6.0, -6.0, 2.5)]):
        r = sc[1:2].copy()
        r[0, :16].view(np.float32)[:] = [x, rad, z, rad]
        extra.append(r)
    sc = np.concatenate([sc] + extra)
    W, H = 40, 24
    rci = oracle.render_call_info(2, W, H)
    for rng_mode in (STREAM, HASH):
        ra, ro, rst = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=rng_mode))
        for accel in (LBVH, GRID, LBVH_OCT, BRUTE):
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, rng_mode=rng_mode, builder=builder)
            assert renderer.scene_array(8)["n_big"] > 4
            assert_same(a, o, ra, ro)
            assert (st.segments, st.samples) == rst[:2]


@pytest.mark.parametrize("builder", [None, "gpu"])
def test_scene_without_big_spheres(rtvk, renderer, torch, oracle, builder):
    """A scene of small spheres only (no ground): no big sphere, so the segment's exhaustive tests
    run on four inert table records (setup_ray tests the first four unconditionally) that must never
    report a hit. Grid, tree and brute-force walks equal the oracle bit for bit, both streams, host
    and device builds."""
    base = oracle.generate_scene()[4:5]
    recs = []
    for i in range(-5, 6):
        for j in range(-5, 6):
            r = base.copy()
            r[0, :16].view(np.float32)[:] = [float(i) * 0.9, 0.2, float(j) * 0.9, 0.2]
            recs.append(r)
    sc = np.concatenate(recs)
    W, H = 40, 24
    rci = oracle.render_call_info(2, W, H)
    f = rci.view(np.float32)
    f[8:11] = [7.0, 3.0, -6.0]
    f[12:15] = [-7.0, -2.8, 6.0]
    for rng_mode in (STREAM, HASH):
        ra, ro, rst = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=rng_mode))
        for accel in (LBVH, GRID, LBVH_OCT, BRUTE):
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, rng_mode=rng_mode, builder=builder)
            assert renderer.scene_array(8)["n_big"] == 0
            assert_same(a, o, ra, ro)
            assert (st.segments, st.samples) == rst[:2]


@pytest.mark.parametrize("builder", [None, "gpu"])
def test_grid_one_layer_and_layered_forms(rtvk, renderer, torch, oracle, builder):
    """The grid walks have a one-layer form (the grid one cell thick in y: the DDA steps x and z
    only), picked when the scene's grid has one cell row in y, as the canonical scenes' grids have,
    and the general 3D form otherwise. Canonical scene: the one-layer form runs (launch_info
    flat_grid) and equals the oracle and the instrumented build (which always runs the general
    form) bit for bit; a stack of small spheres from y = 0.2 to 4.6: the general form runs and
    equals the oracle. Both streams, host grid (LDS) and device grid (L2)."""
    W, H = 48, 32
    base = oracle.generate_scene()[4:5]
    stack = [oracle.generate_scene()[:1].copy()]   # the ground sphere
    rng = np.random.default_rng(11)
    for k in range(240):
        r = base.copy()
        r[0, :16].view(np.float32)[:] = [rng.uniform(-4, 4), 0.2 + 4.4 * k / 239, rng.uniform(-4, 4), 0.2]
        stack.append(r)
    cases = [(oracle.generate_scene(), True, ((13.0, 2.0, 3.0), (0.0, 0.0, 0.0))),
             (np.concatenate(stack), False, ((9.0, 3.0, -9.0), (0.0, 2.0, 0.0)))]
    for sc, flat, (cam, look) in cases:
        rci = oracle.render_call_info(3, W, H)
        f = rci.view(np.float32)
        f[8:11] = cam
        f[12:15] = [look[k] - cam[k] for k in range(3)]
        for rng_mode in (STREAM, HASH):
            ra, ro, rst = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=rng_mode))
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=GRID, rng_mode=rng_mode, builder=builder)
            info = renderer.launch_info()
            assert info["form"].startswith("grid") and info["flat_grid"] == flat, info
            assert (renderer.scene_array(9)["n"][1] == 1) == flat
            assert_same(a, o, ra, ro)
            assert (st.segments, st.samples) == rst[:2]
            a2, o2, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=GRID, rng_mode=rng_mode, builder=builder,
                                   count=True)
            assert not renderer.launch_info()["flat_grid"]
            assert_same(a2, o2, ra, ro)


@pytest.mark.parametrize("K,builder", [(11, None), (40, "gpu")])
@pytest.mark.parametrize("accel", [LBVH, LBVH_OCT, LBVH_GLOBAL])
def test_forced_regate_equals_oracle(rtvk, renderer, torch, oracle, accel, K, builder):
    """The walks test the AABB gate only for the segment's winner; a winner that fails it is
    recomputed by a wave-cooperative gated brute force (regate_brute, ~1 segment in 7e7 on config
    3). Forced here for every segment (options.reserved[0] bit 1): still the oracle's image bit for
    bit, both streams, host scene (grid / octant tree in LDS) and a device-built 6 404-sphere scene
    (grid / treelet / tree from L2)."""
    W, H, spp = 40, 24, 2
    sc = oracle.generate_scene(0.0, K)
    rci = oracle.render_call_info(spp, W, H)
    for rng in (STREAM, HASH):
        ra, ro, rst = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=rng))
        a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, rng_mode=rng, builder=builder,
                              regate=True)
        assert_same(a, o, ra, ro)
        assert (st.segments, st.samples) == rst[:2]


def test_rows_strip_map(rtvk, renderer, torch, oracle):
    W, H = 40, 30
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(3, W, H)
    fa, fo, _ = oracle.render(sc, rci, W, H)
    rows = np.array([29, 0, 8, 9, 10, 15], np.int32)
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, len(rows), rows=rows)
    assert_same(a, o, fa[rows], fo[rows])


@pytest.mark.parametrize("rng_mode", [COUNTER, HASH])
@pytest.mark.parametrize("accel", [BRUTE, LBVH])
def test_accumulate_and_counter_rng(rtvk, renderer, torch, oracle, rng_mode, accel):
    """Progressive accumulation (accumulate + sample_base) in both counter modes: the second call
    adds samples 2..4 to the float accumulator of the first."""
    W, H = 24, 16
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(3, W, H)
    base, _, _ = oracle.render(sc, oracle.render_call_info(2, W, H), W, H, opts=oracle.options(rng_mode=rng_mode))
    ra, ro, _ = oracle.render(sc, rci, W, H, accum=base,
                              opts=oracle.options(rng_mode=rng_mode, accumulate=1, sample_base=2))
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accum=base, rng_mode=rng_mode, accumulate=True,
                         sample_base=2, accel=accel)
    assert_same(a, o, ra, ro)


@pytest.mark.parametrize("chunks", ["1", "2", "3", "7", "13", "4096"])
def test_hash_chunk_invariance(rtvk, renderer, torch, oracle, chunks):
    """RT_RNG_SAMPLE_HASH: splitting every pixel's 13 samples into 1..13 chunks run by different
    lanes in any order (tuning sample_chunks; 4096 is clamped to spp) gives the oracle's bits, with
    the same segment and sample counts, on a ragged band, twice (the second with the LPT order)."""
    W, H, spp = 77, 45, 13
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(spp, W, H)
    ra, ro, rs = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=HASH))
    with tuned(renderer, sample_chunks=chunks):
        for accel in (LBVH, LBVH, BRUTE):
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, rng_mode=HASH, accel=accel)
            assert_same(a, o, ra, ro)
            assert (st.segments, st.samples) == rs[:2]
            if accel == LBVH:
                assert renderer.launch_info()["chunks"] == min(int(chunks), spp)


@pytest.mark.parametrize("head,tail_pm", [("1", "0"), ("2", "300"), ("5", "500"), ("1", "1"), ("3", "1000")])
def test_hash_head_tail_chunks(rtvk, renderer, torch, oracle, head, tail_pm):
    """RT_RNG_SAMPLE_HASH with the LPT order split into a head (the longest tiles, head_chunks
    chunks per pixel) and a tail (tail_tiles_pm per mille of the tiles, `chunks` = 7 chunks):
    the oracle's bits and counts for every split, from all-head (0 per mille) to all-tail (1000,
    no head), on a ragged band; the first launch has no LPT order (no head), the second has."""
    W, H, spp = 77, 45, 13
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(spp, W, H)
    ra, ro, rs = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=HASH))
    with tuned(renderer, sample_chunks=7, head_chunks=head, tail_tiles_pm=tail_pm):
        for k in range(3):
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, rng_mode=HASH, accel=LBVH, count=k == 2)
            assert_same(a, o, ra, ro)
            assert (st.segments, st.samples) == rs[:2]
            info = renderer.launch_info()
            assert info["chunks"] == 7
            if k > 0:
                assert info["head_chunks"] == (None if tail_pm == "1000" else int(head))


def test_hash_tail_steals(rtvk, renderer, torch, oracle):
    """Tail stealing (rt_kernels.hip steal_tail): one chunk per pixel and fewer units than lanes,
    so the queue is empty at once and lanes whose pixels end early (sky) take halves of the
    samples their wave's busiest lanes have not started. The frame keeps the oracle's bits and
    counts for the grid and brute-force kernels (the instrumented builds count the steals; the
    production builds run the same stealing code); the reference stream never steals."""
    W, H, spp = 40, 24, 400
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(spp, W, H)
    ra, ro, rs = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=HASH), threads=16)
    with tuned(renderer, sample_chunks=1):
        for accel in (LBVH, BRUTE):
            for count in (False, True):
                a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, rng_mode=HASH, accel=accel, count=count)
                assert_same(a, o, ra, ro)
                assert (st.segments, st.samples) == rs[:2]
                assert renderer.launch_info()["chunks"] == 1
            assert renderer.steals() > 0
    gpu_render(rtvk, renderer, torch, sc, oracle.render_call_info(4, W, H), W, H, rng_mode=STREAM, accel=LBVH,
               count=True)
    assert renderer.steals() == 0


@pytest.mark.parametrize("rng_mode", [STREAM, HASH])
def test_host_rt_render_bands(rtvk, oracle, rng_mode):
    """rt_render with 3 contiguous bands (one per GPU in the reference, src/ray_trace.cpp:74-93;
    here band i on device i % n), gathered to device 0 by one RCCL group (device 0's bands go
    straight from its buffers) and copied to the host: equals the one-device frame; then
    accumulate on top."""
    W, H = 32, 20
    sc = oracle.generate_scene()
    rcis = [rtvk.canonical_render_call_info(2, W, H) for _ in range(3)]
    for r, y in zip(rcis, (0, 7, 13)):
        r.offset.y = y
    opt = rtvk.make_options(rng_mode=rng_mode)
    res = rtvk.render(rtvk.generateRandomScene(), rcis, options=opt)
    ra, ro, rs = oracle.render(sc, oracle.render_call_info(2, W, H), W, H, opts=oracle.options(rng_mode=rng_mode))
    assert_same(res.accum, res.rgba8, ra, ro)
    assert (res.stats.segments, res.stats.samples) == rs[:2]
    opt2 = rtvk.make_options(rng_mode=rng_mode, accumulate=True, sample_base=2 if rng_mode else 0)
    res2 = rtvk.render(rtvk.generateRandomScene(), rcis, options=opt2, accum=res.accum)
    ra2, ro2, _ = oracle.render(sc, oracle.render_call_info(2, W, H), W, H, accum=ra,
                                opts=oracle.options(rng_mode=rng_mode, accumulate=1, sample_base=2 if rng_mode else 0))
    assert_same(res2.accum, res2.rgba8, ra2, ro2)


@pytest.mark.parametrize("rng_mode", [STREAM, HASH])
def test_multi_renderer_visible_devices(rtvk, torch, oracle, rng_mode):
    """rt_multi over every visible GPU (up to 8): on a multi-GPU box one RCCL communicator, the
    row-exact strips and every other device's rows sent to device 0 in one RCCL group; on a one-GPU
    box one device holding every row renders straight into the caller's buffers (no communicator).
    Two frames (the second with the LPT order) equal the one-device oracle frame bit for bit, and
    the statistics are summed over the devices. (test_multi_logical_devices runs the N > 1 steps
    on one GPU.)"""
    W, H, spp = 72, 43, 3
    sc = oracle.generate_scene()
    rci_np = oracle.render_call_info(spp, W, H)
    ra, ro, rs = oracle.render(sc, rci_np, W, H, opts=oracle.options(rng_mode=rng_mode))
    with rtvk.MultiRenderer(8) as m:
        assert m.device_count == min(8, torch.cuda.device_count())
        m.set_scene(sc)
        rci = rtvk.RenderCallInfo.from_buffer_copy(rci_np.tobytes())
        for _ in range(2):
            acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0")
            out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda:0")
            m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode))
            torch.cuda.synchronize()
            assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra, ro)
            st = m.stats()
            assert (st.segments, st.samples) == rs[:2]
        info = m.info()
        if m.device_count > 1:   # the frame reached the RCCL group: every device rendered rows
            assert info["rccl_ranks"] == m.device_count and info["launches"] == m.device_count
        else:
            assert info["rccl_ranks"] == 0 and info["launches"] == 1


LOGICAL_W, LOGICAL_H = 48, 1080


@pytest.fixture(scope="module")
def logical_refs(oracle):
    """Oracle frames of the logical-device tests: 48 x 1080 at 2 spp (frame 0) and 2 more samples
    accumulated on top (frame 1), in both streams."""
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(2, LOGICAL_W, LOGICAL_H)
    refs = {}
    for mode in (STREAM, HASH):
        base = 2 if mode != STREAM else 0
        a0, o0, s0 = oracle.render(sc, rci, LOGICAL_W, LOGICAL_H, opts=oracle.options(rng_mode=mode), threads=16)
        a1, o1, _ = oracle.render(sc, rci, LOGICAL_W, LOGICAL_H, accum=a0, threads=16,
                                  opts=oracle.options(rng_mode=mode, accumulate=1, sample_base=base))
        refs[mode] = ((a0, o0, s0), (a1, o1))
    return sc, rci, refs


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("rng_mode", [STREAM, HASH])
def test_multi_logical_devices(rtvk, torch, logical_refs, n, rng_mode):
    """rt_multi's N > 1 frame on one GPU (rt_debug_multi_create_logical): n logical devices with
    their own contexts and streams, the row-exact strips, the send / receive pairs of each RCCL
    group as device copies in the group's order, device 0's stage / band buffer selection, the row
    loads and stores and the one resolve: a plain frame and an accumulating frame on top equal the
    oracle bit for bit (the reference's per-GPU band loop, src/ray_trace.cpp:42-105)."""
    sc, rci_np, refs = logical_refs
    (ra0, ro0, rs0), (ra1, ro1) = refs[rng_mode]
    rci = rtvk.RenderCallInfo.from_buffer_copy(rci_np.tobytes())
    with rtvk.MultiRenderer(n, logical=True) as m:
        assert m.device_count == n and m.info()["rccl_ranks"] == 0
        m.tune(balance=0)
        m.set_scene(sc)
        acc = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.float32, device="cuda:0")
        out = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.uint8, device="cuda:0")
        m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode))
        torch.cuda.synchronize()
        assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra0, ro0)
        parts = m.partition(LOGICAL_H)   # the row-exact strips the frame rendered
        for a, b in zip(parts, rtvk.partition_strips(n, LOGICAL_H)):
            np.testing.assert_array_equal(a, b)
        st = m.stats()
        assert (st.segments, st.samples) == rs0[:2]
        assert m.info()["launches"] == n
        base = 2 if rng_mode != STREAM else 0
        m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode, accumulate=True, sample_base=base))
        torch.cuda.synchronize()
        assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra1, ro1)


@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("rng_mode", [STREAM, HASH])
def test_multi_logical_rccl(rtvk, torch, logical_refs, n, rng_mode):
    """rt_multi's RCCL branch on one GPU (rt_debug_multi_create_logical_rccl): ncclCommInitAll of
    one rank, every group's accumulator transfers issued as grouped ncclSend / ncclRecv of that rank
    to itself (the plan's buffers: bands on the logical devices, stages on device 0); a plain and
    an accumulating frame equal the oracle bit for bit."""
    sc, rci_np, refs = logical_refs
    (ra0, ro0, rs0), (ra1, ro1) = refs[rng_mode]
    rci = rtvk.RenderCallInfo.from_buffer_copy(rci_np.tobytes())
    with rtvk.MultiRenderer(n, logical="rccl") as m:
        assert m.device_count == n and m.info()["rccl_ranks"] == 1
        m.tune(balance=0)
        m.set_scene(sc)
        acc = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.float32, device="cuda:0")
        out = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.uint8, device="cuda:0")
        m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode))
        torch.cuda.synchronize()
        assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra0, ro0)
        assert (m.stats().segments, m.stats().samples) == rs0[:2]
        base = 2 if rng_mode != STREAM else 0
        m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode, accumulate=True, sample_base=base))
        torch.cuda.synchronize()
        assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra1, ro1)


@pytest.mark.parametrize("rng_mode", [STREAM, HASH])
def test_multi_logical_rebalance(rtvk, torch, logical_refs, rng_mode):
    """The balancer's re-deals on 8 logical devices: device times fed every frame (device 0 and 3
    slow, rt_debug_multi_feedback) move rows between the devices' bands (rows maps rewritten,
    buffers grown, the LPT records carried over); every frame, plain and accumulating, stays equal
    to the oracle bit for bit, and the partition always holds every row once."""
    sc, rci_np, refs = logical_refs
    (ra0, ro0, _), (ra1, ro1) = refs[rng_mode]
    rci = rtvk.RenderCallInfo.from_buffer_copy(rci_np.tobytes())
    base = 2 if rng_mode != STREAM else 0
    with rtvk.MultiRenderer(8, logical=True) as m:
        m.set_scene(sc)
        start = rtvk.partition_strips(8, LOGICAL_H)
        acc = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.float32, device="cuda:0")
        out = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.uint8, device="cuda:0")
        m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode))   # sets up the strips
        torch.cuda.synchronize()
        assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra0, ro0)
        for f in range(6):
            parts = m.partition(LOGICAL_H)
            assert sorted(np.concatenate(parts).tolist()) == list(range(LOGICAL_H))
            ms = [float(len(p)) * (1.3 if d in (0, 3) else 1.0) for d, p in enumerate(parts)]
            m.feedback(ms)
            m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode))
            torch.cuda.synchronize()
            assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra0, ro0)
            m.feedback(ms)
            m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode, accumulate=True, sample_base=base))
            torch.cuda.synchronize()
            assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra1, ro1)
        info = m.balance_info()
        assert info["rebalances"] >= 2 and info["rows_moved"] >= 8
        end = m.partition(LOGICAL_H)
        assert len(end[0]) < len(start[0]) and len(end[3]) < len(start[3])


def test_multi_logical_balancer_measured(rtvk, torch, logical_refs):
    """rt_multi's balancer on its own measurements (no fed times): 3 logical devices, 6 frames;
    from the third frame on each reads every device's kernel time and tile-cost row weights of the
    frame two before (rt_launch_ms / rt_launch_row_weights internally) and may re-deal. Every frame
    equals the oracle bit for bit; the partition always holds every row once."""
    sc, rci_np, refs = logical_refs
    (ra0, ro0, _), _ = refs[HASH]
    rci = rtvk.RenderCallInfo.from_buffer_copy(rci_np.tobytes())
    with rtvk.MultiRenderer(3, logical=True) as m:
        m.tune(tolerance=0.0)   # re-deal on any measured gain (times on a shared GPU are uneven)
        m.set_scene(sc)
        acc = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.float32, device="cuda:0")
        out = torch.zeros((LOGICAL_H, LOGICAL_W, 4), dtype=torch.uint8, device="cuda:0")
        for _ in range(6):
            m.render(rci, acc, out, options=rtvk.make_options(rng_mode=HASH))
            torch.cuda.synchronize()
            assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra0, ro0)
            parts = m.partition(LOGICAL_H)
            assert sorted(np.concatenate(parts).tolist()) == list(range(LOGICAL_H))
        assert m.balance_info()["frames"] == 6


def test_multi_tune_rejects_bad_settings(rtvk):
    """rt_debug_multi_tune: blend in (0, 1] (0 would freeze the per-row estimates), lag 1-8 (the
    frames the balancer keeps), unknown keys refused; -1 (None) restores a default."""
    with rtvk.MultiRenderer(2, logical=True) as m:
        for kv in ({"blend": 0.0}, {"lag": 9}, {"nonsense": 1}):
            with pytest.raises(RuntimeError):
                m.tune(**kv)
        m.tune(blend=0.25, lag=8, tolerance=0.01)
        m.tune(blend=None, lag=None, tolerance=None, balance=None)


@pytest.mark.parametrize("rng_mode", [STREAM, HASH])
def test_multi_zero_spp_matches_one_device(rtvk, torch, oracle, rng_mode):
    """samplesPerRenderCall = 0 renders the same bytes at every device count (the
    multi-device resolve used to refuse spp 0 that the one-device frame accepts)."""
    W, H = 24, 40
    sc = oracle.generate_scene()
    rci = rtvk.RenderCallInfo.from_buffer_copy(oracle.render_call_info(0, W, H).tobytes())
    got = []
    for n, logical in ((1, False), (3, True)):
        with rtvk.MultiRenderer(n, logical=logical) as m:
            m.set_scene(sc)
            acc = torch.full((H, W, 4), 3.0, dtype=torch.float32, device="cuda:0")
            out = torch.full((H, W, 4), 9, dtype=torch.uint8, device="cuda:0")
            m.render(rci, acc, out, options=rtvk.make_options(rng_mode=rng_mode))
            torch.cuda.synchronize()
            got.append((acc.cpu().numpy(), out.cpu().numpy()))
    np.testing.assert_array_equal(got[0][0].view(np.uint32), got[1][0].view(np.uint32))
    np.testing.assert_array_equal(got[0][1], got[1][1])


def test_host_rt_render_bands_own_spp(rtvk, oracle):
    """rt_render's bands each carry their own RenderCallInfo (src/ray_trace.cpp:660-676 fills one
    per GPU): bands of different samplesPerRenderCall are each rendered and tonemapped with their
    own spp (round 5 refused them)."""
    W, H = 32, 20
    sc = oracle.generate_scene()
    starts, spps = (0, 7, 13), (2, 3, 1)
    rcis = []
    for y, spp in zip(starts, spps):
        r = rtvk.canonical_render_call_info(spp, W, H)
        r.offset.y = y
        rcis.append(r)
    res = rtvk.render(rtvk.generateRandomScene(), rcis, options=rtvk.make_options(rng_mode=STREAM))
    for i, (y0, spp) in enumerate(zip(starts, spps)):
        y1 = starts[i + 1] if i + 1 < len(starts) else H
        rows = np.arange(y0, y1, dtype=np.uint32)
        ra, ro, _ = oracle.render(sc, oracle.render_call_info(spp, W, H), W, len(rows), rows=rows,
                                  opts=oracle.options(rng_mode=STREAM))
        assert_same(res.accum[y0:y1], res.rgba8[y0:y1], ra, ro)


@pytest.mark.parametrize("rng_mode", [COUNTER, HASH])
def test_multi_renderer_accumulate(rtvk, torch, oracle, rng_mode):
    """rt_multi accumulation adds the frame's samples (sample_base) to what the caller's accum
    buffer holds, at every device count (rt_render_device's semantics for the whole image): into
    the same buffer, into another buffer the caller copied the sum to, and, after the first
    buffers are freed, into a new buffer holding a sum the caller changed. The library keeps no
    pointer to an earlier frame's buffer (the direct frame used to keep reading it)."""
    W, H = 40, 27
    sc = oracle.generate_scene()
    rci_np = oracle.render_call_info(2, W, H)
    rci = rtvk.RenderCallInfo.from_buffer_copy(rci_np.tobytes())

    def pair():
        return (torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0"),
                torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda:0"))

    def check(acc, out, prev, k):
        torch.cuda.synchronize()
        ra, ro, _ = oracle.render(sc, rci_np, W, H, accum=prev, opts=oracle.options(
            rng_mode=rng_mode, accumulate=int(k > 0), sample_base=2 * k))
        assert_same(acc.cpu().numpy(), out.cpu().numpy(), ra, ro)
        return ra

    with rtvk.MultiRenderer(8) as m:
        m.set_scene(sc)
        opt = lambda k: rtvk.make_options(rng_mode=rng_mode, accumulate=k > 0, sample_base=2 * k)   # noqa: E731
        a0, o0 = pair()
        m.render(rci, a0, o0, options=opt(0))
        prev = check(a0, o0, None, 0)
        m.render(rci, a0, o0, options=opt(1))                      # same buffer
        prev = check(a0, o0, prev, 1)
        a1, o1 = pair()
        a1.copy_(a0)                                               # the caller moves the sum
        m.render(rci, a1, o1, options=opt(2))
        prev = check(a1, o1, prev, 2)
        del a0, o0, a1, o1
        torch.cuda.empty_cache()
        a2, o2 = pair()
        changed = (prev * np.float32(0.5)).astype(np.float32)     # a running sum the caller edited
        changed[..., 3] = 1.0
        a2.copy_(torch.from_numpy(changed))
        m.render(rci, a2, o2, options=opt(3))
        check(a2, o2, changed, 3)


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
    for form in (LBVH_LDS1, LBVH_GLOBAL):
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
    for accel in FORMS:
        a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel)
        assert_same(a, o, ra, ro)
    a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH, builder="gpu")
    assert_same(a, o, ra, ro)


@pytest.mark.parametrize("builder", [None, "gpu"])
def test_pinhole_origin_shortcut_and_fallback(rtvk, renderer, torch, oracle, builder):
    """Camera rays start at the camera position itself (lf) when the host proves lf + rx crt + ry cup
    is lf (aperture 0, every lf component nonzero); a camera position with a zero component takes
    the general form. Both equal the oracle bit for bit, both streams, grid and brute force."""
    W, H = 40, 24
    sc = oracle.generate_scene()
    for cam, shortcut in [((13.0, 2.0, 3.0), True), ((0.0, 2.0, 12.0), False), ((9.0, 0.0, -9.0), False),
                          ((-0.0, 3.0, 10.0), False)]:
        rci = oracle.render_call_info(2, W, H)
        f = rci.view(np.float32)
        f[8:11] = cam
        f[12:15] = [-cam[0], 0.5 - cam[1], -cam[2]]
        for rng_mode in (STREAM, HASH):
            ra, ro, _ = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=rng_mode))
            for accel in (LBVH, BRUTE):
                a, o, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, rng_mode=rng_mode,
                                     builder=builder)
                assert renderer.launch_info()["pinhole_origin"] == shortcut, cam
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


@pytest.mark.parametrize("form", [LBVH, LBVH_LDS1])
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
    # spp 0 (a 0-sample frame): the trace kernel's own expression, sum / 0 -> +-inf or NaN, so a
    # positive sum stores 255 and everything else 0 (accepted at every device count)
    renderer.resolve_rgba8(torch.from_numpy(a).cuda(), 0, out)
    torch.cuda.synchronize()
    with np.errstate(divide="ignore", invalid="ignore"):
        x = np.sqrt(a[..., :3] / np.float32(0.0))
    want = np.full(a.shape, 255, np.uint8)
    want[..., :3] = np.where(np.isnan(x), 0, np.where(x > 0, 255, 0)).astype(np.uint8)
    np.testing.assert_array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("reserve", ["0", "100", str(1 << 40)])
def test_chunked_refill_same_image(rtvk, renderer, torch, oracle, reserve):
    """Pixel hand-out by whole tiles (refill_reserve = 0), tiles then single pixels (100), and
    single pixels only (huge reserve) render the same image as the oracle, on a ragged frame
    (width and height not multiples of 8) so tiles with missing pixels go through the tile path."""
    W, H = 203, 117
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(3, W, H)
    ra, ro, rs = oracle.render(sc, rci, W, H)
    rh, oh, rsh = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=HASH))
    with tuned(renderer, refill_reserve=reserve):
        for _ in range(2):   # second launch runs with the LPT hand-out order
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH)
            assert_same(a, o, ra, ro)
            assert (st.segments, st.samples) == (rs[0], rs[1])
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH, rng_mode=HASH)
            assert_same(a, o, rh, oh)
            assert (st.segments, st.samples) == (rsh[0], rsh[1])


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


@pytest.mark.parametrize("rng_mode,resolve", [(STREAM, True), (HASH, True), (HASH, False)])
def test_strips_rccl_world1(rtvk, renderer, torch, oracle, rng_mode, resolve):
    """bench.py's N > 1 path (rtvk.dist.DistributedRenderer: row strips per rank, torch.distributed
    gathers over RCCL, rt_scatter_rows on rank 0, rgba8 resolved from the gathered accumulator by
    rt_resolve_rgba8 — or both images gathered — and the balancer's per-frame exchange: the gloo
    side group beside the NCCL default group, the library's launch timer and row weights) on a
    one-rank NCCL group: four frames, each equal to the one-GPU oracle frame bit for bit."""
    import socket
    import torch.distributed as dist
    from rtvk.dist import DistributedRenderer, hip_assembler, hip_band_renderer, hip_band_timer, hip_resolver
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
        dr = DistributedRenderer(W, H, torch.device("cuda", 0),
                                 hip_band_renderer(renderer, rci, rtvk.make_options(rng_mode=rng_mode)),
                                 hip_assembler(renderer), force_gather=True,
                                 resolve=hip_resolver(renderer, spp) if resolve else None,
                                 timer=hip_band_timer(renderer))
        assert dr.cpu_group is not None and dr.timer is not None
        frames = []
        for _ in range(4):
            acc, out = dr.step()
            torch.cuda.synchronize()
            frames.append((acc.cpu().numpy(), out.cpu().numpy()))
        assert dr.rows_per_rank() == [H] and dr.cost.sum() > 0   # measured, nothing to move at one rank
    finally:
        dist.destroy_process_group()
    ra, ro, _ = oracle.render(sc, oracle.render_call_info(spp, W, H), W, H, opts=oracle.options(rng_mode=rng_mode))
    for acc, out in frames:
        assert_same(acc, out, ra, ro)


@pytest.mark.parametrize("isolate", ["0", "3", "1000000"])
def test_isolated_tiles_same_image(rtvk, renderer, torch, oracle, isolate):
    """Waves starting on the longest-chain tiles that take no further pixels (isolate_tiles,
    including every wave isolated) render the same image as the oracle; the second launch has
    the LPT order the isolation needs."""
    W, H = 136, 72
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(2, W, H)
    ra, ro, _ = oracle.render(sc, rci, W, H)
    with tuned(renderer, isolate_tiles=isolate, refill_reserve=0):
        renderer.set_scene(sc)
        rci_c = rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes())
        for _ in range(2):
            a = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
            o = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
            renderer.render_device(rci_c, a, o, options=rtvk.make_options())
            torch.cuda.synchronize()
            assert_same(a.cpu().numpy(), o.cpu().numpy(), ra, ro)



@pytest.mark.parametrize("W,H,spp,K,form", [(320, 180, 2, 158, 0), (320, 180, 2, 158, 8), (320, 180, 2, 158, 10),
                                             (96, 64, 3, 40, 0), (96, 64, 3, 40, 8)])
def test_treelet_walk_equals_brute(rtvk, renderer, torch, oracle, W, H, spp, K, form):
    """Device-built scenes: the default uniform grid walked from L2 (form 0), the tree's top
    levels staged in LDS as a treelet with subtrees below the cut from L2 (ACCEL_LBVH_TOP, form 8)
    and the all-L2 tree walk (form 10) equal brute force bit for bit, twice each (the second
    launch runs with the LPT order)."""
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
    for rng_mode in (STREAM, HASH):
        ra, ro, rs = oracle.render(sc, rci, W, H, opts=oracle.options(max_depth=depth if depth else 50,
                                                                     rng_mode=rng_mode))
        for accel in (BRUTE, LBVH):
            a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=accel, max_depth=depth,
                                  rng_mode=rng_mode)
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


def test_scene_and_render_on_a_side_stream(rtvk, torch, oracle):
    """set_scene and render_device inside torch.cuda.stream(s) (a non-blocking stream): the upload
    is ordered before the render on s, and a render issued next on the default stream is ordered
    after it (the context chains its operations across streams)."""
    W, H = 64, 40
    scs = [oracle.generate_scene(t) for t in (0.0, 1.3)]
    rci = oracle.render_call_info(2, W, H)
    rci_c = rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes())
    with rtvk.Renderer(0) as r:
        s = torch.cuda.Stream()
        accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(3)]
        outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(3)]
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            r.set_scene(scs[0])
            r.render_device(rci_c, accs[0], outs[0], options=rtvk.make_options())
            r.set_scene(scs[1])
            r.render_device(rci_c, accs[1], outs[1], options=rtvk.make_options(rng_mode=HASH))
        r.render_device(rci_c, accs[2], outs[2], options=rtvk.make_options())   # default stream
        torch.cuda.synchronize()
        for k, (sc, mode) in enumerate([(scs[0], STREAM), (scs[1], HASH), (scs[1], STREAM)]):
            ra, ro, _ = oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=mode))
            assert_same(accs[k].cpu().numpy(), outs[k].cpu().numpy(), ra, ro)


def test_render_streams_alternate_on_one_context(rtvk, torch, oracle):
    """Back-to-back renders of one context on different streams share its work counters and LPT
    tables; the second waits for the first, so neither frame loses or repeats pixels."""
    W, H = 160, 96
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(3, W, H)
    rci_c = rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes())
    ra, ro, _ = oracle.render(sc, rci, W, H)
    with rtvk.Renderer(0) as r:
        r.set_scene(sc)
        streams = [torch.cuda.Stream() for _ in range(2)]
        bufs = [(torch.zeros((H, W, 4), dtype=torch.float32, device="cuda"),
                 torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")) for _ in range(4)]
        torch.cuda.synchronize()
        for k, (a, o) in enumerate(bufs):
            r.render_device(rci_c, a, o, options=rtvk.make_options(), stream=streams[k % 2])
        torch.cuda.synchronize()
        for a, o in bufs:
            assert_same(a.cpu().numpy(), o.cpu().numpy(), ra, ro)


@pytest.mark.parametrize("refit", [False, True])
def test_device_build_between_streams(rtvk, torch, oracle, refit):
    """A render on stream A, then a device-built scene (its build runs on the context's build
    stream beside the render), then a render on stream B: the second render must
    wait for the first one too (it reuses the context's counters, tile costs and big-sphere table),
    not only for the build. Both frames equal the oracle's; then the same with the
    streams swapped."""
    W, H, spp = 128, 64, 1024   # frame 0 runs ~1 ms on the GPU: longer than the build beside it
    scs = [oracle.generate_scene(t) for t in (0.0, 0.7, 1.9)]
    rci = oracle.render_call_info(spp, W, H)
    rci_c = rtvk.RenderCallInfo.from_buffer_copy(rci.tobytes())
    refs = [oracle.render(sc, rci, W, H, opts=oracle.options(rng_mode=HASH), threads=16)[:2] for sc in scs]
    with rtvk.Renderer(0) as r:
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        bufs = [(torch.zeros((H, W, 4), dtype=torch.float32, device="cuda"),
                 torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")) for _ in range(3)]
        dev_scs = [torch.from_numpy(sc).cuda() for sc in scs]
        torch.cuda.synchronize()
        opt = rtvk.make_options(rng_mode=HASH, accel=LBVH)
        r.set_scene_device(dev_scs[0], stream=sa)
        r.render_device(rci_c, *bufs[0], options=opt, stream=sa)
        r.set_scene_device(dev_scs[1], refit=refit, stream=sa)       # build beside frame 0
        r.render_device(rci_c, *bufs[1], options=opt, stream=sb)    # frame 1 on the other stream
        r.set_scene_device(dev_scs[2], refit=refit, stream=sb)
        r.render_device(rci_c, *bufs[2], options=opt, stream=sa)
        torch.cuda.synchronize()
        assert r.scene_array(8)["device_built"]
        for (a, o), (ra, ro) in zip(bufs, refs):
            assert_same(a.cpu().numpy(), o.cpu().numpy(), ra, ro)


def test_render_before_scene_fails(rtvk, torch):
    with rtvk.Renderer(0) as r:
        acc = torch.zeros((8, 8, 4), dtype=torch.float32, device="cuda")
        out = torch.zeros((8, 8, 4), dtype=torch.uint8, device="cuda")
        with pytest.raises(rtvk.RtError) as e:
            r.render_device(rtvk.canonical_render_call_info(1, 8, 8), acc, out)
        assert e.value.code == -4   # RT_ERR_NO_SCENE
        r.set_scene(np.zeros((0, 80), np.uint8))   # an empty scene is a scene (sky only)
        r.render_device(rtvk.canonical_render_call_info(1, 8, 8), acc, out)
        torch.cuda.synchronize()


def test_scatter_rows_bounds(rtvk, renderer, torch):
    """Row maps pointing past the destination are refused by the Python mirror and skipped by the
    kernel (dst_rows bound), never written out of bounds."""
    W = 16
    src_a = torch.ones((3, W, 4), dtype=torch.float32, device="cuda")
    src_o = torch.full((3, W, 4), 9, dtype=torch.uint8, device="cuda")
    dst_a = torch.zeros((4, W, 4), dtype=torch.float32, device="cuda")
    dst_o = torch.zeros((4, W, 4), dtype=torch.uint8, device="cuda")
    bad = torch.tensor([0, 4, 2], dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        renderer.scatter_rows(src_a, src_o, bad, dst_a, dst_o)
    # straight through the C-ABI: row 4 of a 4-row destination is skipped
    guard = torch.zeros((5, W, 4), dtype=torch.uint8, device="cuda")   # row 4 = canary
    from rtvk import abi
    abi.check(rtvk.load_library().rt_scatter_rows(renderer._ctx, src_a.data_ptr(), src_o.data_ptr(), bad.data_ptr(),
                                                  3, W, 4, None, guard.data_ptr(), None))
    torch.cuda.synchronize()
    g = guard.cpu().numpy()
    assert (g[0] == 9).all() and (g[2] == 9).all() and (g[1] == 0).all() and (g[3] == 0).all() and (g[4] == 0).all()


# ---- BASELINE configs 3 and 5 at their own workloads ------------------------------------------
def test_config3_full_frame(rtvk, renderer, torch, oracle):
    """BASELINE config 3 in full: 1920x1080, 10 000 spp, LBVH + persistent threads, the reference
    stream (~2 s on one MI355X). Four evenly spaced 4x16-pixel blocks are rendered by the oracle at
    the same 10 000 spp and must match bit for bit; the whole frame must be finite and lit."""
    W, H, spp = 1920, 1080, 10000
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(spp, W, H)
    a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH)
    assert st.samples == W * H * spp
    assert np.isfinite(a).all() and (a[..., 3] == 1.0).all() and o[..., :3].mean() > 40
    for y in (67, 403, 740, 1013):   # 16 rows x 4 pixels: one oracle thread per row
        rows = np.arange(y, y + 16, dtype=np.uint32)
        r = oracle.render_call_info(spp, W, H, (896, 0))
        ra, ro, _ = oracle.render(sc, r, 4, 16, rows=rows, threads=16)
        assert_same(a[y:y + 16, 896:900], o[y:y + 16, 896:900], ra, ro)


def test_config3_hash_full_frame(rtvk, renderer, torch, oracle):
    """Config 3's workload in RT_RNG_SAMPLE_HASH mode (the bench's headline stream): two 4x16-pixel
    blocks against the oracle, bit for bit, and the frame agrees with the reference-stream
    frame statistically (two independent 10 000-spp estimates of one picture: PSNR >= 40 dB)."""
    W, H, spp = 1920, 1080, 10000
    sc = oracle.generate_scene()
    rci = oracle.render_call_info(spp, W, H)
    a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH, rng_mode=HASH)
    assert st.samples == W * H * spp and renderer.launch_info()["chunks"] >= 1
    for y in (211, 877):
        r = oracle.render_call_info(spp, W, H, (1200, 0))
        ra, ro, _ = oracle.render(sc, r, 4, 16, rows=np.arange(y, y + 16, dtype=np.uint32),
                                  opts=oracle.options(rng_mode=HASH), threads=16)
        assert_same(a[y:y + 16, 1200:1204], o[y:y + 16, 1200:1204], ra, ro)
    a_ref, o_ref, _ = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH)
    mse = np.mean((o[..., :3].astype(np.float64) - o_ref[..., :3]) ** 2)
    assert 10 * np.log10(255 ** 2 / mse) >= 40.0


def test_config5_full_frame(rtvk, renderer, torch, oracle):
    """BASELINE config 5 on one GPU: 3840x2160, 99 860 spheres (the reference recipe with a
    316x316 grid), 1 000 spp. The production walk (uniform grid from L2), the treelet walk (LDS
    treelet + L2 subtrees) and the all-L2 tree walk agree bit for bit with the same segment counts,
    and a 4x16-pixel block at an offset
    matches the oracle (brute force over all 99 860 spheres) at the full 1 000 spp."""
    W, H, spp, K = 3840, 2160, 1000, 158
    sc = oracle.generate_scene(0.0, K)
    rci = oracle.render_call_info(spp, W, H)
    a, o, st = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=LBVH, rng_mode=HASH)
    assert renderer.launch_info()["form"] == "grid-global" and renderer.launch_info()["flat_grid"]
    for form in (LBVH_OCT, LBVH_GLOBAL):   # the treelet walk and the all-L2 tree walk
        a2, o2, st2 = gpu_render(rtvk, renderer, torch, sc, rci, W, H, accel=form, rng_mode=HASH)
        assert_same(a, o, a2, o2)
        assert (st.segments, st.samples) == (st2.segments, st2.samples) and st.samples == W * H * spp
    r = oracle.render_call_info(spp, W, H, (1800, 0))
    ra, ro, _ = oracle.render(sc, r, 4, 16, rows=np.arange(1200, 1216, dtype=np.uint32),
                              opts=oracle.options(rng_mode=HASH), threads=16)
    assert_same(a[1200:1216, 1800:1804], o[1200:1216, 1800:1804], ra, ro)


def test_reference_image_qualitative(rtvk, torch):
    """Qualitative pin against the reference's only rendered output (sceneRender.png, README.md:3;
    statistics in tests/golden/sceneRender_stats.npz). That image is not a pixel oracle: its scene
    layout differs from the generator's (no camera or scene time reproduces it, thumbnail PSNR
    <= 17 dB over a sweep), and its spp is unknown. The upstream view (shader.rgen:29, camera
    (13, 2, -3) -> origin) rendered at 1920x1080 must still agree in what the shading decides:
    the sky blocks exactly, per-channel means within 6 %, per-channel 32-bin histograms within
    L1 0.3 (measured: 1.4 / 3.5 / 4.1 % and 0.21 / 0.21 / 0.23)."""
    import sys
    sys.path.insert(0, str(GOLDEN))
    from make_scene_render_ref import stats
    W, H = 1920, 1080
    rci = rtvk.canonical_render_call_info(256, W, H)
    rci.camera_pos.x, rci.camera_pos.y, rci.camera_pos.z = 13.0, 2.0, -3.0
    rci.camera_dir.x, rci.camera_dir.y, rci.camera_dir.z = -13.0, -2.0, 3.0
    with rtvk.Renderer(0) as r:
        r.set_scene(rtvk.generateRandomScene())
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        r.render_device(rci, acc, out, options=rtvk.make_options(rng_mode=HASH))
        torch.cuda.synchronize()
    ours = stats(out.cpu().numpy()[..., :3])
    ref = np.load(GOLDEN / "sceneRender_stats.npz", allow_pickle=False)
    np.testing.assert_allclose(np.median(ours["thumb"][:3].reshape(-1, 3), axis=0),
                               np.median(ref["thumb"][:3].reshape(-1, 3), axis=0), atol=0.5)
    m_ours, m_ref = ours["thumb"].mean(axis=(0, 1)), ref["thumb"].mean(axis=(0, 1))
    assert (np.abs(m_ours / m_ref - 1) < 0.06).all(), (m_ours, m_ref)
    assert (np.abs(ours["hist"] - ref["hist"]).sum(axis=1) < 0.3).all()


@pytest.mark.parametrize("accel", [BRUTE, LBVH])
def test_checkered_dielectric_and_odd_materials(rtvk, renderer, torch, oracle, accel):
    """Material records outside the generator's recipe: a checkered dielectric (its colors[1] is
    the checker's, so the kernel computes eta and r0 itself instead of reading the record's
    precomputed constants), a fuzzy metal, a diffuse sphere with the checker, an unknown material
    id (no scatter: its colour is light), all against the oracle in both random stream modes."""
    sc = oracle.generate_scene()
    recs = sc.copy()
    f, u = recs.view(np.float32).reshape(-1, 20), recs.view(np.uint32).reshape(-1, 20)
    u[3, 5] = 1                                     # big glass sphere: checkered
    f[3, 12:16] = [0.9, 0.2, 0.3, 1.0]              # its colors[1]
    u[2, 4], f[2, 16] = 1, 0.35                     # big metal: fuzz 0.35 (scene.h leaves 0)
    u[1, 5] = 1                                     # big diffuse sphere: checkered
    f[1, 12:16] = [0.1, 0.8, 0.2, 1.0]
    u[10, 4] = 7                                    # unknown material id
    W, H = 96, 54
    rci = oracle.render_call_info(3, W, H)
    for mode in (STREAM, HASH):
        ra, ro, rs = oracle.render(recs, rci, W, H, opts=oracle.options(rng_mode=mode))
        a, o, st = gpu_render(rtvk, renderer, torch, recs, rci, W, H, accel=accel, rng_mode=mode)
        assert_same(a, o, ra, ro)
        assert (st.segments, st.samples) == rs[:2]
