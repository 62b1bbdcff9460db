"""Diagnostic (RT_LIB selects a library build): predicted strong-scaling of the multi-GPU frame from one GPU. For N GPUs, rank 0
renders the 8-row strips k = 0 mod N (rtvk.dist.strip_rows); this times that band alone (after a
warm-up launch, so the LPT hand-out is in effect) and reports N x its Msamples/s against the
full frame, plus the launch telemetry (queue dry / tail). Mode `samples` times rank 0's share of
a sample-split frame instead (the full frame at spp/N samples)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402
from rtvk.dist import split_samples, strip_rows  # noqa: E402

W, H = 1920, 1080
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
walk = int(sys.argv[2]) if len(sys.argv) > 2 else 0
mode = sys.argv[3] if len(sys.argv) > 3 else "strips"   # strips | samples
lib = abi.load_library()
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
rci = rtvk.canonical_render_call_info(spp, W, H)
opt = rtvk.make_options(accel=2)
opt.reserved[1] = walk
print(f"library: {os.environ.get('RT_LIB', abi.LIB_PATH)}")
for _ in range(1):
  base = None
  for n in (1, 2, 4, 8):
      rows_np = strip_rows(0, n, H) if mode == "strips" else np.arange(H, dtype=np.int32)
      if mode == "samples":   # rank 0's share of a sample-split frame: the full frame at spp/N
          rci = rtvk.canonical_render_call_info(split_samples(spp, n)[0], W, H)
      rows = torch.from_numpy(rows_np).cuda()
      acc = torch.zeros((len(rows_np), W, 4), dtype=torch.float32, device="cuda")
      out = torch.zeros((len(rows_np), W, 4), dtype=torch.uint8, device="cuda")
      ts, tails, runs = [], [], []
      for i in range(5):
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
      v = W * len(rows_np) * rci.samplesPerRenderCall / ms / 1e3 * n
      if base is None:
          base = v
      print(f"N={n}: band {len(rows_np)} rows, {ms:.2f} ms, queue {np.median(runs):.2f} ms, tail {np.median(tails):.2f} ms -> "
            f"{v:.0f} Msamples/s if every rank matched rank 0 (efficiency vs linear: {v / (base * n):.2f})",
            flush=True)
