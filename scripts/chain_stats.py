"""Diagnostic: per-pixel chain lengths (traced segments of the longest pixel of every 8x8 tile,
recorded by the trace kernel for the LPT hand-out) on the canonical 1080p frame."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H = 1920, 1080
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
lib = abi.load_library()
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
r.render_device(rtvk.canonical_render_call_info(spp, W, H), acc, out, options=rtvk.make_options(accel=2))
torch.cuda.synchronize()
n = ctypes.c_uint64()
abi.check(lib.rt_debug_tile_cost(r._ctx, None, 0, ctypes.byref(n)))
c = (ctypes.c_uint32 * n.value)()
abi.check(lib.rt_debug_tile_cost(r._ctx, c, n.value, ctypes.byref(n)))
c = np.array(c, np.float64)
st = r.stats()
print(f"spp {spp}: mean segments/pixel {st.segments / (W * H):.0f}; tile max-chain: mean {c.mean():.0f}, "
      f"p50 {np.percentile(c, 50):.0f}, p90 {np.percentile(c, 90):.0f}, p99 {np.percentile(c, 99):.0f}, "
      f"p99.9 {np.percentile(c, 99.9):.0f}, max {c.max():.0f}")
