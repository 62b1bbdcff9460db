"""Diagnostic: SIMD placement of the trace kernel's waves (a -DRT_PLACEMENT build), for every
variant library given: waves per SIMD over the chip and the histogram of a block's busiest SIMD.
Usage: python scripts/placement.py lib1.so [lib2.so ...]"""
import ctypes
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

W, H, spp = 1920, 1080, 20
scene = rtvk.generateRandomScene()
rci = rtvk.canonical_render_call_info(spp, W, H)
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
for lp in sys.argv[1:]:
    lib = abi.load_library(lp)
    ctx = ctypes.c_void_p()
    assert lib.rt_context_create(0, ctypes.byref(ctx)) == 0
    assert lib.rt_set_scene(ctx, ctypes.addressof(scene), len(scene), None) == 0
    for walk in (8, 6):
        opt = rtvk.make_options(accel=2, rng_mode=rtvk.HASH)
        opt.reserved[1] = walk
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert lib.rt_render_device(ctx, ctypes.byref(rci), None, W, H, acc.data_ptr(), out.data_ptr(),
                                    ctypes.byref(opt), torch.cuda.current_stream().cuda_stream) == 0
        e1.record()
        torch.cuda.synchronize()
        u = (ctypes.c_uint64 * 32)()
        assert lib.rt_debug_util(ctx, u) == 0
        li = (ctypes.c_uint32 * 4)()
        lib.rt_debug_launch_info(ctx, li)
        hist = {m - 8: u[m] for m in range(8, 32) if u[m]}
        print(f"{lp.split('/')[-1]:<22} walk {walk}: {e0.elapsed_time(e1):7.2f} ms  lds {li[2]}  waves per SIMD "
              f"{[u[k] for k in range(4)]}  blocks by busiest-SIMD waves {hist}", flush=True)
