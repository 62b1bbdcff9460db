import sys, ctypes
sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch, rtvk
from rtvk import abi
r = rtvk.Renderer(0); sc = rtvk.generateRandomScene(); r.set_scene(sc)
for spp, W, H in [(8, 1920, 1080)]:
    rci = rtvk.canonical_render_call_info(spp, W, H)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda"); out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    for md in (50, 1, 2):
        r.render_device(rci, acc, out, options=rtvk.make_options(accel=2, count_tests=True, max_depth=md)); torch.cuda.synchronize()
        st = r.stats(); s8 = (ctypes.c_uint64 * 8)(); abi.load_library().rt_debug_stamps(r._ctx, s8)
        print(f"max_depth {md}: segs {st.segments} box/seg {st.box_tests/st.segments:.2f} sph/seg {st.sphere_tests/st.segments:.2f} wave_iters {s8[6]} util {st.box_tests/(64*s8[6]):.3f}")
