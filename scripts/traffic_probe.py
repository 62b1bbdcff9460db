#!/usr/bin/env python3
"""One frame of the hot path for a rocprofv3 --pmc pass (HBM traffic of the trace + resolve
kernels): warm-up frame, then the measured frame. Environment knobs of the library (e.g.
RT_TILE_TAIL) apply. Usage: python scripts/traffic_probe.py [spp] [W H K] [rng: hash|stream]"""
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
W, H, K = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080, 11)
rng = rtvk.STREAM if (sys.argv[5] if len(sys.argv) > 5 else "hash") == "stream" else rtvk.HASH
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene(0.0, K))
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, W, H)
for _ in range(2):
    r.render_device(rci, acc, out, options=rtvk.make_options(rng_mode=rng))
torch.cuda.synchronize()
print("ok", r.launch_info(), r.kernel_times(2))
