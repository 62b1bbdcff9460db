"""One canonical frame (plus a warm-up frame) through a given library build, for rocprofv3 --pmc
A/B of variants (bench.py refuses alternative libraries). usage:
python scripts/frame_once.py LIB.so [spp=100] [W=1920 H=1080 K=11] [rng=2]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))
import torch  # noqa: E402

import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

lib = sys.argv[1]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 100
W, H, K = (int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (1920, 1080, 11)
rng = int(sys.argv[6]) if len(sys.argv) > 6 else 2
abi.load_library(lib)
abi._lib = abi.load_library(lib)   # rtvk's calls go to this build
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene(0.0, K))
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, W, H)
opt = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=rng)
for _ in range(2):
    r.render_device(rci, acc, out, options=opt)
torch.cuda.synchronize()
print("frames ok", lib, r.kernel_times(2))
r.close()
