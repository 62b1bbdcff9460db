#!/usr/bin/env python3
"""A/B of the uniform grid's cell scale (tuning grid_scale, rt_grid.h kGridCellScale) on the
config 3 frame, interleaved rounds in one process. The scale is applied when the scene is built, so
every timed render follows its own set_scene (outside the timed region); every scale must render
the same image. Usage: python scripts/grid_scale_ab.py SPP ROUNDS scale [scale ...] [--config5]
(--config5: config 5's frame, 3840x2160 and the 99 860-sphere scene, grid built on the device)."""
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

c5 = "--config5" in sys.argv
argv = [a for a in sys.argv if a != "--config5"]
spp, rounds = int(argv[1]), int(argv[2])
scales = [float(x) for x in argv[3:]]
W, H = (3840, 2160) if c5 else (1920, 1080)
r = rtvk.Renderer(0)
scene = rtvk.generateRandomScene(0.0, 158 if c5 else 11)
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, W, H)
opts = rtvk.make_options(rng_mode=rtvk.HASH)
times = {s: [] for s in scales}
forms = {}
ref = None
for rnd in range(rounds + 1):
    for s in scales:
        r.tune(grid_scale=s)
        r.set_scene(scene)
        r.render_device(rci, acc, out, options=opts)   # LPT history of this scale's tiles
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render_device(rci, acc, out, options=opts)
        e1.record()
        torch.cuda.synchronize()
        forms[s] = r.launch_info()["form"]
        if rnd == 0:
            img = acc.cpu().numpy()
            if ref is None:
                ref = img
            assert np.array_equal(img, ref), f"scale {s} changed the image"
        else:
            times[s].append(e0.elapsed_time(e1))
r.tune(grid_scale=None)
base = np.median(times[scales[0]])
print(f"{'config 5 ' if c5 else ''}spp {spp}, {rounds} rounds: " + ", ".join(
    f"scale {s} [{forms[s]}] {np.median(v):.2f} ms ({(np.median(v) / base - 1) * 100:+.2f} %, min {min(v):.2f})"
    for s, v in times.items()), flush=True)
