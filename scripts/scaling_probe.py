"""Diagnostic (RT_LIB selects a library build): predicted strong scaling of the multi-GPU frame
from one GPU. For N GPUs, rank r renders the 8-row strips k = r mod N (rtvk.dist.strip_rows);
this times rank r's band alone for every r (after a warm-up launch, so the LPT hand-out is in
effect) and reports the frame time max_r(band time) against the one-GPU frame, plus the launch
telemetry of rank 0 (work queue dry / tail after it).

usage: python scripts/scaling_probe.py [spp] [rng: hash|stream] [N list, e.g. 1,2,4,8]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402
from rtvk.dist import strip_rows  # noqa: E402

W, H = 1920, 1080
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
rng = rtvk.HASH if (sys.argv[2] if len(sys.argv) > 2 else "hash") == "hash" else rtvk.STREAM
ns = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,8").split(",")]
lib = abi.load_library()
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
rci = rtvk.canonical_render_call_info(spp, W, H)
opt = rtvk.make_options(accel=2, rng_mode=rng)
print(f"library: {os.environ.get('RT_LIB', abi.LIB_PATH)}  spp {spp}  rng {'hash' if rng == rtvk.HASH else 'stream'}")
base = None
for n in ns:
    worst, first = 0.0, None
    for rank in range(n):
        rows_np = strip_rows(rank, n, H)
        rows = torch.from_numpy(rows_np).cuda()
        acc = torch.zeros((len(rows_np), W, 4), dtype=torch.float32, device="cuda")
        out = torch.zeros((len(rows_np), W, 4), dtype=torch.uint8, device="cuda")
        ts, tails, runs = [], [], []
        for i in range(3 if spp >= 1000 else 5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.render_device(rci, acc, out, rows=rows, options=opt)
            e1.record()
            torch.cuda.synchronize()
            h = (ctypes.c_uint64 * 68)()
            abi.check(lib.rt_debug_lane_hist(r._ctx, h))
            if i:
                ts.append(e0.elapsed_time(e1))
                tails.append((h[67] - h[66]) / 1e5)
                runs.append((h[66] - h[65]) / 1e5)
        ms = float(np.median(ts))
        worst = max(worst, ms)
        if first is None:
            first = (ms, float(np.median(runs)), float(np.median(tails)), r.launch_info()["chunks"])
        if spp >= 1000 and n == 8 and rank >= 1:   # bands of one N are alike: rank 0 and 1 suffice
            break
    v = W * H * spp / worst / 1e3
    if base is None:
        base = v * ns[0]
    print(f"N={n}: slowest band {worst:.2f} ms (rank 0: {first[0]:.2f} ms, queue {first[1]:.2f} ms, tail "
          f"{first[2]:.2f} ms, {first[3]} chunks/pixel) -> {v:.0f} Msamples/s, efficiency vs linear "
          f"{v / (base * n):.3f}", flush=True)
