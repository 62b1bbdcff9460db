#!/usr/bin/env python3
"""A/B: the same frame with and without a rows map (the strip tiling's band-row -> global-row map
that every N > 1 launch passes; an identity map here), interleaved rounds, images must agree.
Usage: python scripts/rows_map_ab.py [spp] [rng: hash|stream]"""
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
rng = rtvk.STREAM if (sys.argv[2] if len(sys.argv) > 2 else "hash") == "stream" else rtvk.HASH
W, H = 1920, 1080
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
rci = rtvk.canonical_render_call_info(spp, W, H)
rows = torch.arange(H, dtype=torch.int32, device="cuda")
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
times = {"none": [], "identity": []}
ref = None
for rnd in range(4):
    for k, m in (("none", None), ("identity", rows)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render_device(rci, acc, out, rows=m, options=rtvk.make_options(rng_mode=rng))
        e1.record()
        torch.cuda.synchronize()
        if rnd == 0:
            img = acc.cpu().numpy()
            ref = img if ref is None else ref
            assert np.array_equal(img, ref)
        else:
            times[k].append(e0.elapsed_time(e1))
print(f"spp {spp}: " + ", ".join(f"rows {k} {np.median(v):.2f} ms" for k, v in times.items()))
