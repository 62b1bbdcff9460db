#!/usr/bin/env python3
"""A/B of the grid's cell scale (RT_GRID_SCALE, read when the scene is set) in one process,
interleaved rounds; every scale must render the same image. Usage:
  python scripts/scale_ab.py spp scale [scale ...]   (AB_W / AB_H / AB_K: frame, scene)"""
import os
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

W, H, K = int(os.environ.get("AB_W", 1920)), int(os.environ.get("AB_H", 1080)), int(os.environ.get("AB_K", 11))
spp, scales = int(sys.argv[1]), sys.argv[2:]
scene = rtvk.generateRandomScene(0.0, K)
rci = rtvk.canonical_render_call_info(spp, W, H)
opt = rtvk.make_options(accel=rtvk.abi.RT_ACCEL_AUTO, rng_mode=rtvk.HASH)
rs = {}
for sc in scales:   # one context per scale: the grid is built at set_scene
    rs[sc] = rtvk.Renderer(0)
    rs[sc].tune(grid_scale=float(sc))
    rs[sc].set_scene(scene)
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
times, ref = {s: [] for s in scales}, None
for rnd in range(4):
    for sc in scales:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rs[sc].render_device(rci, acc, out, options=opt)
        e1.record()
        torch.cuda.synchronize()
        if rnd == 0:
            img = acc.cpu().numpy()
            ref = img if ref is None else ref
            assert np.array_equal(img, ref), f"scale {sc} differs"
        else:
            times[sc].append(e0.elapsed_time(e1))
print(f"{W}x{H} K={K} spp {spp}: " + ", ".join(f"scale {s} {np.median(t):.2f} ms" for s, t in times.items()), flush=True)
