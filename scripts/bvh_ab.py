"""A/B of the tree builders (RT_BVH_BUILD=gpu|morton|sah, RT_SAH_KNOBS) on a 1080p frame.

Usage: python scripts/bvh_ab.py [grid_half_extent [spp [builder:knobs/builder:knobs...]]]

Prints per builder: box / sphere tests per segment and walk SIMD utilisation (instrumented
build, 8 spp), then the kernel time of the 100-spp frame (HIP events, median of 5).
Both trees give bit-identical images; the check at the end asserts it.
"""
import ctypes
import os
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H = 1920, 1080
grid = int(sys.argv[1]) if len(sys.argv) > 1 else 11
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 100
r = rtvk.Renderer(0)
sc = rtvk.generateRandomScene(grid_half_extent=grid) if grid != 11 else rtvk.generateRandomScene()
images = {}
combos = [("gpu", ""), ("morton", ""), ("sah", ""), ("sah", "classic"), ("sah", "sweep"),
          ("sah", "order1"), ("sah", "order2")]
if len(sys.argv) > 3:
    combos = [tuple((c + ":").split(":")[:2]) for c in sys.argv[3].split("/")]
for builder, knobs in combos:
    os.environ["RT_BVH_BUILD"] = builder
    r.tune(sah_knobs=(1 if "classic" in knobs else 0) | (2 if "sweep" in knobs else 0)
           | (4 if "order1" in knobs else 8 if "order2" in knobs else 0))
    r.set_scene(sc)
    torch.cuda.synchronize()
    rci8 = rtvk.canonical_render_call_info(8, W, H)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    r.render_device(rci8, acc, out, options=rtvk.make_options(accel=2, count_tests=True))
    torch.cuda.synchronize()
    st = r.stats()
    s8 = (ctypes.c_uint64 * 8)()
    abi.load_library().rt_debug_stamps(r._ctx, s8)
    util = st.box_tests / (64 * s8[6]) if s8[6] else float("nan")
    rci = rtvk.canonical_render_call_info(spp, W, H)
    opts = rtvk.make_options(accel=2)
    ts = []
    for i in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render_device(rci, acc, out, options=opts)
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    ts.sort()
    images[(builder, knobs)] = out.cpu()
    print(f"{builder:7s} {knobs:14s} grid {grid}: box/seg {st.box_tests / st.segments:.2f} "
          f"sph/seg {st.sphere_tests / st.segments:.2f} walk util {util:.3f} "
          f"frame {ts[len(ts) // 2]:.2f} ms ({spp} spp)", flush=True)
first = next(iter(images.values()))
assert all(torch.equal(first, v) for v in images.values()), "builders disagree"
print("images identical")
