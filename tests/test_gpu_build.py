"""Device LBVH build / refit (rt_build.hip) against the host builder (rt_bvh.cpp) and the oracle.

The device builder is specified to emit exactly the host builder's tree (Morton form), so every
scene array is compared bit for bit (node boxes as floats, so -0.0 == +0.0; links and counts as
integers). Refit results are checked through rendering against the CPU oracle (bit-exact), since
any valid topology renders the identical image.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import LBVH, assert_same, tree_builder

pytestmark = pytest.mark.gpu


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


def scene_arrays(renderer):
    out = {k: renderer.scene_array(k) for k in range(8) if k != 5}
    out["info"] = renderer.scene_array(8)
    return out


def build_both(renderer, spheres):
    with tree_builder("morton"):   # the host form the device builder reproduces
        renderer.set_scene(spheres)
        host = scene_arrays(renderer)
        host[5] = renderer.scene_array(5)
    with tree_builder("gpu"):
        renderer.set_scene(spheres)
        dev = scene_arrays(renderer)
        dev[5] = renderer.scene_array(5)
    return host, dev


def nodes_equal(a, b):
    a, b = np.asarray(a).reshape(-1, 32), np.asarray(b).reshape(-1, 32)
    assert a.shape == b.shape
    fa, fb = a.view(np.float32), b.view(np.float32)
    ua, ub = a.view(np.uint32), b.view(np.uint32)
    box = [0, 1, 2, 4, 5, 6]
    np.testing.assert_array_equal(fa[:, box], fb[:, box])   # -0.0 == +0.0
    np.testing.assert_array_equal(ua[:, [3, 7]], ub[:, [3, 7]])   # escape, first_count


def assert_trees_equal(host, dev):
    hi, di = host["info"], dev["info"]
    assert not hi["device_built"] and di["device_built"]
    for k in ("n_spheres", "n_big", "n_nodes", "n_leaf", "small_rmax", "scene_radius"):
        assert hi[k] == di[k], (k, hi[k], di[k])
    for k in (0, 1, 2, 3, 6, 7):
        np.testing.assert_array_equal(host[k].view(np.uint8), dev[k].view(np.uint8), err_msg=f"array {k}")
    nodes_equal(host[4], dev[4])
    nodes_equal(host[5], dev[5])


def records(oracle, centers, radii, t=0.0):
    """(n, 80) sphere records: canonical materials cycled, given geometry."""
    base = oracle.generate_scene(t, 11)
    n = len(radii)
    rec = np.ascontiguousarray(base[np.arange(n) % len(base)].copy())
    g = np.zeros((n, 4), np.float32)
    g[:, :3] = centers
    g[:, 3] = radii
    rec[:, :16] = g.view(np.uint8).reshape(n, 16)
    return rec


@pytest.mark.parametrize("t,K", [(0.0, 11), (1.3, 11), (0.0, 1), (0.0, 2), (0.5, 40), (0.0, 158), (0.0, 363)])
def test_device_tree_equals_host_tree(renderer, oracle, t, K):
    sc = oracle.generate_scene(t, K)
    host, dev = build_both(renderer, sc)
    assert dev["info"]["n_nodes"] > 0
    assert_trees_equal(host, dev)


@pytest.mark.parametrize("case", ["one", "two", "five", "dups", "all_equal", "many_big", "flat_line"])
def test_device_tree_edge_cases(renderer, oracle, case):
    rng = np.random.default_rng(7)
    if case == "one":
        c, r = np.array([[0, -1000, 1]], np.float32), np.array([1000], np.float32)
    elif case == "two":
        c, r = np.array([[0, -1000, 1], [1, 0.2, 1]], np.float32), np.array([1000, 0.2], np.float32)
    elif case == "five":
        c = rng.uniform(-3, 3, (5, 3)).astype(np.float32)
        r = np.full(5, 0.2, np.float32)
    elif case == "dups":   # coincident centers: equal Morton codes, position-augmented split
        c = np.repeat(rng.uniform(-5, 5, (37, 3)).astype(np.float32), 7, axis=0)
        r = rng.uniform(0.1, 0.3, len(c)).astype(np.float32)
    elif case == "all_equal":   # every center identical: zero extent on every axis
        c = np.zeros((33, 3), np.float32)
        r = np.full(33, 0.5, np.float32)
    elif case == "many_big":   # > 64 spheres above 2 x median, with tied radii
        c = rng.uniform(-50, 50, (300, 3)).astype(np.float32)
        r = np.concatenate([np.full(200, 0.2), rng.choice([3.0, 4.0, 5.0], 100)]).astype(np.float32)
    else:   # all centers on a line: one axis spans, the others are flat
        c = np.zeros((129, 3), np.float32)
        c[:, 0] = np.linspace(-10, 10, 129)
        r = np.full(129, 0.05, np.float32)
    host, dev = build_both(renderer, records(oracle, c, r))
    assert_trees_equal(host, dev)


@pytest.mark.parametrize("n", [126, 127, 128, 129, 130, 4095, 4097, 8193, 8320])
def test_device_tree_box_pyramid_sizes(renderer, oracle, n):
    """Node boxes and cut-tree counts come from a pyramid of 64-sphere unions (rt_build.hip
    k_nodebox): scenes whose small-sphere counts straddle the pyramid's group and range limits
    (128 entries read whole, 64-aligned splits, 64^2 groups) build the host tree bit for bit. K = 363
    above (527 080 spheres) reaches the pyramid's top level."""
    rng = np.random.default_rng(n)
    c = rng.uniform(-20, 20, (n, 3)).astype(np.float32)
    c[:, 1] = rng.uniform(0, 0.5, n)
    r = rng.uniform(0.05, 0.25, n).astype(np.float32)
    host, dev = build_both(renderer, records(oracle, c, r))
    assert_trees_equal(host, dev)


@pytest.mark.parametrize("K,device_built,form", [(11, False, "grid-lds-rec"), (15, False, "grid-lds"),
                                                 (16, True, "lbvh-octant-lds"), (40, True, "grid-global"),
                                                 (158, True, "grid-global")])
def test_auto_builder_policy(renderer, oracle, K, device_built, form):
    """Default: host SAH tree up to 1024 spheres (K = 15 -> 904), device LBVH above (K = 16 ->
    1028); the walk is the uniform grid over the small spheres staged in LDS (host-built scenes;
    with the shading records too while two blocks per CU still fit, K = 11),
    else the tree's 8 octant copies in LDS while they fit (K = 16), else the grid from L2
    (device-built scenes, K = 40 -> 6404)."""
    with tree_builder(None):
        os.environ.pop("RT_BVH_BUILD", None)
        renderer.set_scene(oracle.generate_scene(0.0, K))
    assert renderer.scene_array(8)["device_built"] == device_built
    assert renderer.launch_info()["form"] == form


def test_empty_scene_device_build(renderer):
    with tree_builder("gpu"):
        renderer.set_scene(np.zeros((0, 80), np.uint8))
    info = renderer.scene_array(8)
    assert info["n_spheres"] == 0 and info["n_nodes"] == 0 and info["device_built"]


def render_small(rtvk, renderer, torch, oracle, spheres_for_oracle, W=48, H=32, spp=3):
    rci_u32 = oracle.render_call_info(spp, W, H, (0, 0))
    rci = rtvk.RenderCallInfo.from_buffer_copy(np.ascontiguousarray(rci_u32).tobytes())
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    renderer.render_device(rci, acc, out, options=rtvk.make_options(accel=LBVH))
    torch.cuda.synchronize()
    a_ref, o_ref, _ = oracle.render(spheres_for_oracle, rci_u32, W, H, threads=8)
    assert_same(acc.cpu().numpy(), out.cpu().numpy(), a_ref, o_ref)


def test_refit_animation_frames(rtvk, renderer, torch, oracle):
    """Reference animation (spheres 1-3 move with t): build at t=0, refit per frame."""
    with tree_builder("gpu"):
        renderer.set_scene(oracle.generate_scene(0.0, 11))
        nodes0 = renderer.scene_array(4)
        for t in (0.4, 1.7):
            sc = oracle.generate_scene(t, 11)
            renderer.refit_scene(sc)
            assert renderer.scene_array(8)["device_built"]
            render_small(rtvk, renderer, torch, oracle, sc)
        # the moving spheres are outside the tree: its nodes equal a fresh build's
        renderer.set_scene(oracle.generate_scene(1.7, 11))
        nodes_equal(nodes0, renderer.scene_array(4))


def test_refit_moved_small_spheres(rtvk, renderer, torch, oracle):
    """Tree spheres move and grow: the refit tree keeps the old topology, the image stays exact."""
    rng = np.random.default_rng(3)
    sc = oracle.generate_scene(0.0, 11)
    with tree_builder("gpu"):
        renderer.set_scene(sc)
        moved = sc.copy()
        g = moved[:, :16].copy().view(np.float32).reshape(-1, 4)
        g[4:, 0] += rng.uniform(-0.8, 0.8, len(g) - 4).astype(np.float32)
        g[4:, 2] += rng.uniform(-0.8, 0.8, len(g) - 4).astype(np.float32)
        g[4:, 3] *= np.float32(1.5)
        moved[:, :16] = g.view(np.uint8).reshape(-1, 16)
        renderer.refit_scene(moved)
        info = renderer.scene_array(8)
        assert info["small_rmax"] == pytest.approx(0.3)
        render_small(rtvk, renderer, torch, oracle, moved)


def test_refit_keeps_device_memory(rtvk, renderer, torch, oracle):
    """Every refit of a device-built scene rebuilds its uniform grid; the previous grid's arrays
    are released (they once leaked, ~1 MB per refit here), and the image stays exact."""
    sc = oracle.generate_scene(0.0, 40)   # 6 404 spheres: device build + grid from L2
    with tree_builder("gpu"):
        renderer.set_scene(sc)
        renderer.refit_scene(sc)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        for t in (0.3, 0.6, 0.9) * 10:
            renderer.refit_scene(oracle.generate_scene(t, 40))
        torch.cuda.synchronize()
        assert free0 - torch.cuda.mem_get_info()[0] < 4 << 20
        sc = oracle.generate_scene(0.9, 40)
        renderer.refit_scene(sc)
        render_small(rtvk, renderer, torch, oracle, sc)


def test_set_scene_device_input(rtvk, renderer, torch, oracle):
    sc = oracle.generate_scene(0.25, 11)
    with tree_builder("gpu"):
        renderer.set_scene(sc)
        ref = scene_arrays(renderer)
    renderer.set_scene_device(torch.from_numpy(sc).cuda())
    dev = scene_arrays(renderer)
    for k in (0, 1, 2, 3, 4, 6, 7):
        np.testing.assert_array_equal(ref[k].view(np.uint8), dev[k].view(np.uint8))
    renderer.set_scene_device(torch.from_numpy(oracle.generate_scene(0.9, 11)).cuda(), refit=True)
    render_small(rtvk, renderer, torch, oracle, oracle.generate_scene(0.9, 11))


def test_far_camera_repad_device_tree(rtvk, renderer, torch, oracle):
    """A camera beyond the padded radius re-pads the device tree from its unpadded boxes."""
    sc = oracle.generate_scene(0.0, 11)
    with tree_builder("gpu"):
        renderer.set_scene(sc)
    raw = renderer.scene_array(5)
    W, H = 40, 24
    rci_u32 = oracle.render_call_info(2, W, H, (0, 0))
    rci_u32 = rci_u32.copy()
    f = rci_u32.view(np.float32)
    f[8:11] = np.array([13e4, 11e4, -3e4], np.float32)       # camera_pos far away
    f[12:15] = np.array([-13e4, -11e4, 3e4], np.float32)     # looking at the scene
    rci = rtvk.RenderCallInfo.from_buffer_copy(rci_u32.tobytes())
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    renderer.render_device(rci, acc, out, options=rtvk.make_options(accel=LBVH))
    torch.cuda.synchronize()
    a_ref, o_ref, _ = oracle.render(sc, rci_u32, W, H, threads=8)
    assert_same(acc.cpu().numpy(), out.cpu().numpy(), a_ref, o_ref)
    nodes_equal(raw, renderer.scene_array(5))   # the unpadded copy is untouched
    padded = renderer.scene_array(4).view(np.float32).reshape(-1, 8)
    assert (padded[:, 0] < raw.view(np.float32).reshape(-1, 8)[:, 0]).all()
