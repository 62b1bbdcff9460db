"""Diagnostic: tail-compaction pool A/B on the canonical 1080p frame (walk option 7 = pool,
default = the LDS-scene kernel without it). Frame time from HIP events, plus the
launch telemetry: when the pixel queue ran dry and how long the tail after it took. Images must
be identical. Extra libraries (build variants) may be passed as arguments."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H, spp = 1920, 1080, 100
libs = [str(abi.LIB_PATH)] + sys.argv[1:]
scene = rtvk.generateRandomScene()
rci = rtvk.canonical_render_call_info(spp, W, H)
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()
ctxs = []
for lp in libs:
    lib = abi.load_library(lp)
    ctx = ctypes.c_void_p()
    assert lib.rt_context_create(0, ctypes.byref(ctx)) == 0
    assert lib.rt_set_scene(ctx, ctypes.addressof(scene), len(scene), None) == 0
    ctxs.append((lp.split("/")[-1], lib, ctx))
ref = None
for rep in range(2):
    for name, lib, ctx in ctxs:
        for walk in (0, 7):
            opt = rtvk.make_options(accel=2)
            opt.reserved[1] = walk
            ts, drys, tails = [], [], []
            for i in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                assert lib.rt_render_device(ctx, ctypes.byref(rci), None, W, H, acc.data_ptr(), out.data_ptr(),
                                            ctypes.byref(opt), stream.cuda_stream) == 0
                e1.record(stream)
                torch.cuda.synchronize()
                h = (ctypes.c_uint64 * 68)()
                assert lib.rt_debug_lane_hist(ctx, h) == 0
                if i:
                    ts.append(e0.elapsed_time(e1))
                    drys.append((h[66] - h[65]) / 1e5)
                    tails.append((h[67] - h[66]) / 1e5)
            img = out.cpu()
            if ref is None:
                ref = img
            assert torch.equal(ref, img), (name, walk)
            print(f"{name:24s} walk {walk}: frame {np.median(ts):.2f} ms (min {min(ts):.2f}), queue dry at "
                  f"{np.median(drys):.2f} ms, tail {np.median(tails):.2f} ms", flush=True)
print("images identical")
