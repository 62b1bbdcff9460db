"""Diagnostic: LBVH walks of several library builds against brute force on the bench frame
(1920x1080, 100 spp): differing pixels per build and walk form."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H, spp = 1920, 1080, int(sys.argv[1]) if len(sys.argv) > 1 else 100
scene = rtvk.generateRandomScene()
rci = rtvk.canonical_render_call_info(spp, W, H)
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()
ref = None
for lp in [str(abi.LIB_PATH)] + sys.argv[2:]:
    lib = abi.load_library(lp)
    ctx = ctypes.c_void_p()
    assert lib.rt_context_create(0, ctypes.byref(ctx)) == 0
    assert lib.rt_set_scene(ctx, ctypes.addressof(scene), len(scene), None) == 0
    for accel, walk in ((1, 0), (2, 0), (2, 8)):
        opt = rtvk.make_options(accel=accel)
        opt.reserved[1] = walk
        assert lib.rt_render_device(ctx, ctypes.byref(rci), None, W, H, acc.data_ptr(), out.data_ptr(),
                                    ctypes.byref(opt), stream.cuda_stream) == 0
        torch.cuda.synchronize()
        img = acc.cpu().numpy()
        if ref is None:
            ref = img
        bad = np.argwhere(np.any(img != ref, axis=-1))
        print(f"{lp.split('/')[-1]:20s} accel {accel} walk {walk}: {len(bad)} pixels differ from brute "
              f"force {bad[:6].tolist()}", flush=True)
