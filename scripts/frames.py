"""Renders K frames of the canonical 1080p scene at S spp (profiling driver, no checks).
Usage: python scripts/frames.py [spp] [frames]"""
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 12
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
acc = torch.zeros((1080, 1920, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((1080, 1920, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, 1920, 1080)
for _ in range(k):
    r.render_device(rci, acc, out, options=rtvk.make_options())
torch.cuda.synchronize()
print("ok", flush=True)
