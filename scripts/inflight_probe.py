#!/usr/bin/env python3
"""Diagnostic: frames in flight. K frames of the canonical 1080p scene (per-frame rebuild +
render), with F contexts/streams used round robin so frame k+1's blocks can start on the CUs
frame k's tail leaves idle. Prints ms per frame for F = 1, 2, 3 and checks every frame's image
equals the F = 1 image. Usage: python scripts/inflight_probe.py [spp] [frames]"""
import sys
import time

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
W, H = 1920, 1080
scene = rtvk.generateRandomScene()
rci = rtvk.canonical_render_call_info(spp, W, H)
ref = None
for F in (1, 2, 3):
    rs = [rtvk.Renderer(0) for _ in range(F)]
    ss = [torch.cuda.Stream() for _ in range(F)]
    acc = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(F)]
    out = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(F)]

    def frame(k):
        i = k % F
        rs[i].set_scene(scene, stream=ss[i])
        rs[i].render_device(rci, acc[i], out[i], options=rtvk.make_options(), stream=ss[i])

    for k in range(2 * F):   # warm-up: every context has its LPT order
        frame(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        frame(k)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    imgs = [a.cpu().numpy() for a in acc]
    if ref is None:
        ref = imgs[0]
    assert all(np.array_equal(im, ref) for im in imgs), "frames in flight changed the image"
    print(f"spp {spp} frames in flight {F}: {ms:.2f} ms/frame -> {W * H * spp / ms / 1e3:.0f} Msamples/s",
          flush=True)
    for r in rs:
        r.close()
