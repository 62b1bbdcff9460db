#!/usr/bin/env python3
"""Walk-length histogram (box tests per segment, hit vs miss) of the LBVH kernel, 1080p."""
import ctypes
import json
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
W, H, spp = 1920, 1080, int(sys.argv[1]) if len(sys.argv) > 1 else 8
rci = rtvk.canonical_render_call_info(spp, W, H)
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
for md in (50, 1):
    r.render_device(rci, acc, out, options=rtvk.make_options(accel=2, count_tests=True, max_depth=md))
    torch.cuda.synchronize()
    h = (ctypes.c_uint64 * 128)()
    abi.check(abi.load_library().rt_debug_walk_hist(r._ctx, h))
    h = np.array(h, dtype=np.float64).reshape(2, 64)
    tot = h.sum()
    mean = [(h[k] * np.arange(64)).sum() / max(1, h[k].sum()) for k in (0, 1)]
    print(json.dumps({"max_depth": md, "miss_frac": round(h[0].sum() / tot, 4), "mean_miss": round(mean[0], 2),
                      "mean_hit": round(mean[1], 2), "miss_hist": h[0].astype(int).tolist(),
                      "hit_hist": h[1].astype(int).tolist()}))
