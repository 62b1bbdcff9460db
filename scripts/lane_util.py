"""Diagnostic: lane utilisation per kernel code point (RT_UTIL build) of the canonical frame.
Build:  make -C ray-tracing-gpu-vulkan_amd variant NAME=util VFLAGS=-DRT_UTIL
Run:    RT_LIB=ray-tracing-gpu-vulkan_amd/lib/variants/librt_util.so python scripts/lane_util.py [spp] [W H K]

For each point: wave passes, mean active lanes of 64 (utilisation while the point executes), and
the point's share of all counted lane-slots (passes x 64), a proxy for its share of issue time
weighted by the instructions each pass costs (the cost column is a static VALU estimate)."""
import ctypes
import os
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
W, H, K = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080, 11)
NAMES = {0: "node visit (LDS)", 11: "node visit (L2)", 1: "leaf test", 2: "sphere candidate", 8: "segment (tracing)",
         7: "sample start", 3: "shade", 10: "shade hit", 9: "unit vector", 4: "diffuse", 5: "metal",
         6: "dielectric", 12: "node pass <=8 lanes", 13: "node pass <=16", 14: "node pass <=32"}
r = rtvk.Renderer(0)


def opts(rng):
    """Walk form from RT_WALK (options.reserved[1]: 8 octant tree, 12 grid; default 0)."""
    o = rtvk.make_options(accel=2, rng_mode=rng)
    o.reserved[1] = int(os.environ.get("RT_WALK", "0"))
    return o


r.set_scene(rtvk.generateRandomScene(0.0, K))
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, W, H)
lib = abi.load_library()
for rng in (rtvk.HASH,):
    r.render_device(rci, acc, out, options=opts(rng))
    torch.cuda.synchronize()
    u = (ctypes.c_uint64 * 32)()
    abi.check(lib.rt_debug_util(r._ctx, u))
    st = r.stats()
    print(f"{W}x{H} spp {spp} grid {K} rng {'hash' if rng == rtvk.HASH else 'stream'}: segments {st.segments}")
    if os.environ.get("RT_WALK", "0") in ("0", "12"):   # grid walks: slots 12-15 describe test1's candidates
        NAMES.update({12: "cand beyond best", 13: "cand = winner", 14: "cand < tmin", 15: "cand pass, none useful"})
    for k in (8, 7, 0, 12, 13, 14, 15, 11, 1, 2, 3, 10, 9, 4, 5, 6):
        n, a = u[2 * k], u[2 * k + 1]
        if n == 0:
            continue
        print(f"  {k:2d} {NAMES[k]:<18} passes {n:14d}  per segment {n * 64 / max(1, st.segments):7.3f}  "
              f"mean lanes {a / n:6.2f} / 64  util {a / n / 64:.3f}")
