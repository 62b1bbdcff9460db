"""Walk work of primary (depth 0) vs bounce segments in the default grid walk (COUNT build).

Per segment pass: the wave's walk work (cells + reference tests) max over all tracing lanes and
over bounce lanes only. (all - bounce) / all bounds what a cheaper primary walk could save in wave
passes of the walk. Usage: python scripts/walk_split.py [spp]
"""
import ctypes
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402

import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 1920, 1080
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
rci = rtvk.canonical_render_call_info(spp, W, H)
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
lib = abi.load_library()
for rng, name in ((rtvk.HASH, "hash"), (rtvk.STREAM, "stream")):
    r.render_device(rci, acc, out, options=rtvk.make_options(rng_mode=rng, count_tests=True))
    torch.cuda.synchronize()
    st = r.stats()
    v = (ctypes.c_uint64 * 4)()
    abi.check(lib.rt_debug_walk_split(r._ctx, v))
    allw, bw, pw, pn = list(v)
    print(f"{name}: segs {st.segments} primary segs {pn} ({pn / st.segments:.3f}); "
          f"walk work/primary seg {pw / max(pn, 1):.2f}; wave walk passes all {allw} bounce-only {bw} "
          f"-> primary-bound share {(allw - bw) / max(allw, 1):.3f}", flush=True)
