"""Diagnostic: persistent-kernel tail by pixel hand-out order on the canonical 1080p frame:
row-major, tiles by total cost (RT_SCHEDULE=sum), tiles by longest pixel chain (default, "lpt"). Reports frame time and the launch telemetry:
when the pixel queue ran dry and how long the tail after it took. Images must be identical."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H = 1920, 1080
RNG = rtvk.HASH if os.environ.get("AB_RNG", "stream") == "hash" else rtvk.STREAM   # AB_RNG=hash
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
lib = abi.load_library()
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, W, H)
imgs = {}
for rep in range(3):
    for mode in ("rowmajor", "sum", "lpt"):
        r.tune(schedule={"lpt": 0, "rowmajor": 1, "sum": 2}[mode])
        ts, tails, drys = [], [], []
        for i in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.render_device(rci, acc, out, options=rtvk.make_options(accel=2, rng_mode=RNG))
            e1.record()
            torch.cuda.synchronize()
            h = (ctypes.c_uint64 * 68)()
            abi.check(lib.rt_debug_lane_hist(r._ctx, h))
            if i:
                ts.append(e0.elapsed_time(e1))
                drys.append((h[66] - h[65]) / 1e5)
                tails.append((h[67] - h[66]) / 1e5)
        imgs[mode] = out.cpu()
        print(f"{mode:8s}: frame {np.median(ts):.2f} ms (min {min(ts):.2f}), queue dry at "
              f"{np.median(drys):.2f} ms, tail {np.median(tails):.2f} ms", flush=True)
assert all(torch.equal(imgs["rowmajor"], v) for v in imgs.values())
print("images identical")
