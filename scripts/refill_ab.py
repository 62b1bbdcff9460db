#!/usr/bin/env python3
"""A/B of the pixel hand-out (RT_REFILL_RESERVE, read per launch) in one process, interleaved:
`off` = pixel-by-pixel refill everywhere, `lane` = default (tiles until one pixel per lane is
left), `0` = tiles to the end. Full 1080p frames at several spp; every setting must give the
same image. Usage: python scripts/refill_ab.py [spp ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

W, H = 1920, 1080
spps = [int(a) for a in sys.argv[1:] if "=" not in a] or [13, 25, 100]
settings = {"off": str(1 << 40), "lane": None, "0": "0"}
for a in sys.argv[1:]:   # name=reserve adds a setting
    if "=" in a:
        k, v = a.split("=")
        settings[k] = v
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
for spp in spps:
    rci = rtvk.canonical_render_call_info(spp, W, H)
    times = {k: [] for k in settings}
    ref = None
    for rnd in range(5):
        for k, v in settings.items():
            r.tune(refill_reserve=None if v is None else float(v))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.render_device(rci, acc, out, options=rtvk.make_options())
            e1.record()
            torch.cuda.synchronize()
            if rnd == 0:
                img = acc.cpu().numpy()
                if ref is None:
                    ref = img
                assert np.array_equal(img, ref), f"refill setting {k} changed the image"
            else:
                times[k].append(e0.elapsed_time(e1))
    print(f"spp {spp}: " + ", ".join(f"{k} {np.median(v):.2f} ms" for k, v in times.items()), flush=True)
