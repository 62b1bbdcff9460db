"""Diagnostic: per-pixel chain lengths (traced segments of the longest pixel of every 8x8 tile,
recorded by the trace kernel for the LPT hand-out) on the canonical 1080p frame, against the
launch time and its queue / tail split: is the frame bound by its longest chain?
Usage: python scripts/chain_stats.py [spp ...]"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H = 1920, 1080
lib = abi.load_library()
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
for spp in [int(a) for a in sys.argv[1:]] or [100]:
    ts, qs, tl = [], [], []
    for i in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render_device(rtvk.canonical_render_call_info(spp, W, H), acc, out, options=rtvk.make_options(accel=2))
        e1.record()
        torch.cuda.synchronize()
        h = (ctypes.c_uint64 * 68)()
        abi.check(lib.rt_debug_lane_hist(r._ctx, h))
        if i:
            ts.append(e0.elapsed_time(e1))
            qs.append((h[66] - h[65]) / 1e5)
            tl.append((h[67] - h[66]) / 1e5)
    n = ctypes.c_uint64()
    abi.check(lib.rt_debug_tile_cost(r._ctx, None, 0, ctypes.byref(n)))
    c = (ctypes.c_uint32 * n.value)()
    abi.check(lib.rt_debug_tile_cost(r._ctx, c, n.value, ctypes.byref(n)))
    c = np.array(c, np.float64)
    st = r.stats()
    ms = float(np.median(ts))
    print(f"spp {spp}: {ms:.2f} ms (queue {np.median(qs):.2f}, tail {np.median(tl):.2f}); mean segments/pixel "
          f"{st.segments / (W * H):.0f}; tile max-chain: mean {c.mean():.0f}, p50 {np.percentile(c, 50):.0f}, "
          f"p99 {np.percentile(c, 99):.0f}, p99.9 {np.percentile(c, 99.9):.0f}, max {c.max():.0f} -> "
          f"{ms * 1e3 / c.max():.2f} us per segment of the longest chain", flush=True)
