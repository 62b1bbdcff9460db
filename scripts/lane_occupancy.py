"""Diagnostic: persistent-kernel lane occupancy (segment-loop iterations by tracing lanes) of the
canonical 1080p frame, from the instrumented build (rt_debug_lane_hist)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H = 1920, 1080
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = rtvk.HASH if len(sys.argv) > 2 and sys.argv[2] == "hash" else rtvk.STREAM   # usage: [spp] [hash|stream]
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
r.render_device(rtvk.canonical_render_call_info(spp, W, H), acc, out,
                options=rtvk.make_options(rng_mode=rng, count_tests=True))
torch.cuda.synchronize()
h = (ctypes.c_uint64 * 68)()
abi.check(abi.load_library().rt_debug_lane_hist(r._ctx, h))
t0, tdry, tend = h[65], h[66], h[67]
h = np.array(h[:65], np.float64)
k = np.arange(65)
iters = h.sum()
print(f"spp {spp}: segment-loop iterations {iters:.0f}, mean tracing lanes {np.dot(h, k) / iters:.2f} / 64 "
      f"(occupancy {np.dot(h, k) / iters / 64:.3f})")
for lo, hi in [(0, 16), (16, 32), (32, 48), (48, 60), (60, 65)]:
    sel = slice(lo, hi)
    print(f"  {lo:2d}-{hi - 1:2d} lanes: {h[sel].sum() / iters * 100:5.1f} % of iterations, "
          f"{np.dot(h[sel], k[sel]) / np.dot(h, k) * 100:5.1f} % of lane-segments")
r.render_device(rtvk.canonical_render_call_info(spp, W, H), acc, out, options=rtvk.make_options(rng_mode=rng))
torch.cuda.synchronize()
h2 = (ctypes.c_uint64 * 68)()
abi.check(abi.load_library().rt_debug_lane_hist(r._ctx, h2))
t0, tdry, tend = h2[65], h2[66], h2[67]
print(f"  production kernel: span {(tend - t0) / 1e5:.2f} ms (100 MHz clock); pixel queue dry at "
      f"{(tdry - t0) / 1e5:.2f} ms; tail after dry {(tend - tdry) / 1e5:.2f} ms "
      f"({(tend - tdry) / (tend - t0) * 100:.1f} %)")
