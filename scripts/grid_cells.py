#!/usr/bin/env python3
"""Empty visited cells of the grid walks (COUNT build, rt_debug_grid_cells): the share of DDA steps
whose cell holds no reference — the decision metric of an occupancy bitmap. BASELINE
configs 3 (grid in LDS) and 5 (device grid from L2), hash stream.
Usage: python scripts/grid_cells.py [spp3 spp5]"""
import json
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

spp3, spp5 = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (100, 20)
res = {}
for name, (W, H, spp, K) in {"config3": (1920, 1080, spp3, 11), "config5": (3840, 2160, spp5, 158)}.items():
    r = rtvk.Renderer(0)
    r.set_scene(rtvk.generateRandomScene(0.0, K))
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    r.render_device(rtvk.canonical_render_call_info(spp, W, H), acc, out,
                    options=rtvk.make_options(rng_mode=rtvk.HASH, count_tests=True))
    torch.cuda.synchronize()
    c, st = r.grid_cells(), r.stats()
    res[name] = {"spp": spp, "form": r.launch_info()["form"], "cells": c["cells"], "empty": c["empty"],
                 "empty_share": round(c["empty"] / max(1, c["cells"]), 4),
                 "cells_per_segment": round(c["cells"] / max(1, st.segments), 3),
                 "refs_per_segment": round(st.sphere_tests / max(1, st.segments), 3)}
    r.close()
print(json.dumps(res, indent=1))
