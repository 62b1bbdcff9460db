#!/usr/bin/env python3
"""A/B of a per-launch tuning knob (rt_debug_tune; names as RT_SAMPLE_CHUNKS or sample_chunks) in one
process, interleaved rounds, full 1080p frames: every setting must render the same image. Usage:
  python scripts/env_ab.py KNOB spp[,spp...] name=value [name=value ...]   (value '-' = default)"""
import os
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

W, H = int(os.environ.get("AB_W", 1920)), int(os.environ.get("AB_H", 1080))   # AB_W / AB_H / AB_K: frame, scene
RNG = rtvk.HASH if os.environ.get("AB_RNG", "stream") == "hash" else rtvk.STREAM   # AB_RNG=hash
var = sys.argv[1]
key = var[3:].lower() if var.startswith("RT_") else var
spps = [int(x) for x in sys.argv[2].split(",")]
settings = dict(a.split("=", 1) for a in sys.argv[3:])
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene(0.0, int(os.environ.get("AB_K", 11))))
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
for spp in spps:
    rci = rtvk.canonical_render_call_info(spp, W, H)
    times = {k: [] for k in settings}
    ref = None
    for rnd in range(6):
        for k, v in settings.items():
            r.tune(**{key: None if v == "-" else float(v)})
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.render_device(rci, acc, out, options=rtvk.make_options(rng_mode=RNG))
            e1.record()
            torch.cuda.synchronize()
            if rnd == 0:
                img = acc.cpu().numpy()
                if ref is None:
                    ref = img
                assert np.array_equal(img, ref), f"{var}={v} changed the image"
            else:
                times[k].append(e0.elapsed_time(e1))
    print(f"spp {spp}: " + ", ".join(f"{k} {np.median(v):.2f} ms" for k, v in times.items()), flush=True)
