#!/usr/bin/env python3
"""A/B of several per-launch environment settings in one process, interleaved rounds, on the
config 3 frame (or AB_W x AB_H, AB_K grid): every setting must render the same image. Usage:
  python scripts/envs_ab.py SPP ROUNDS name=VAR:value[,VAR:value...] ...   (value '-' = unset)"""
import os
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

W, H = int(os.environ.get("AB_W", 1920)), int(os.environ.get("AB_H", 1080))
RNG = rtvk.STREAM if os.environ.get("AB_RNG", "hash") == "stream" else rtvk.HASH
spp, rounds = int(sys.argv[1]), int(sys.argv[2])
settings = {}
for a in sys.argv[3:]:
    name, kv = a.split("=", 1)
    settings[name] = [tuple(x.split(":", 1)) for x in kv.split(",") if x]
knobs = sorted({k for v in settings.values() for k, _ in v})
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene(0.0, int(os.environ.get("AB_K", 11))))
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, W, H)
times = {k: [] for k in settings}
ref = None
for rnd in range(rounds + 1):
    for name, kvs in settings.items():
        r.tune(**{(k[3:].lower() if k.startswith("RT_") else k): None for k in knobs})   # rt_debug_tune
        r.tune(**{(k[3:].lower() if k.startswith("RT_") else k): (None if v == "-" else float(v)) for k, v in kvs})
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render_device(rci, acc, out, options=rtvk.make_options(rng_mode=RNG))
        e1.record()
        torch.cuda.synchronize()
        if rnd == 0:
            img = acc.cpu().numpy()
            if ref is None:
                ref = img
            assert np.array_equal(img, ref), f"{name} changed the image"
        else:
            times[name].append(e0.elapsed_time(e1))
base = np.median(next(iter(times.values())))
print(f"spp {spp}, {rounds} rounds: " + ", ".join(
    f"{k} {np.median(v):.2f} ms ({(np.median(v) / base - 1) * 100:+.2f} %, min {min(v):.2f})" for k, v in times.items()),
    flush=True)
