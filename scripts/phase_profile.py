"""Diagnostic: where a trace launch's wave time goes, from a -DRT_STAMPS build (per-wave s_memtime
phase stamps summed into Counters::stamp, rt_debug_stamps). Build it with
  make -C ray-tracing-gpu-vulkan_amd variant NAME=stamps VFLAGS=-DRT_STAMPS
and run RT_LIB=ray-tracing-gpu-vulkan_amd/lib/variants/librt_stamps.so python scripts/phase_profile.py [spp] [rng]

Phases (rt_kernels.hip lbvh_loop): 0 loop head (ballots, refill call), 4 sample start (camera ray,
seed), 5 refill (unit hand-out), 6 block fetch (atomic + tile seeds), 1 ray setup (reciprocals, big
spheres), 2 LBVH walk, 3 shading, 7 other (exit)."""
import ctypes
import os
import sys

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 200
rng = rtvk.HASH if (sys.argv[2] if len(sys.argv) > 2 else "hash") == "hash" else rtvk.STREAM
W, H, K = (int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (1920, 1080, 11)
r = rtvk.Renderer(0)


def opts(rng):
    """Walk form from RT_WALK (options.reserved[1]: 8 octant tree, 12 grid; default 0)."""
    o = rtvk.make_options(accel=2, rng_mode=rng)
    o.reserved[1] = int(os.environ.get("RT_WALK", "0"))
    return o


r.set_scene(rtvk.generateRandomScene(0.0, K))
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
rci = rtvk.canonical_render_call_info(spp, W, H)
names = {0: "loop head", 4: "sample start", 5: "refill", 6: "block fetch", 1: "ray setup", 2: "walk", 3: "shading",
         7: "other"}
for i in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r.render_device(rci, acc, out, options=opts(rng))
    e1.record()
    torch.cuda.synchronize()
st = (ctypes.c_uint64 * 8)()
abi.check(abi.load_library().rt_debug_stamps(r._ctx, st))
tot = sum(st)
print(f"spp {spp} rng {'hash' if rng == rtvk.HASH else 'stream'}: {e0.elapsed_time(e1):.2f} ms (stamped build)")
for k in (0, 4, 5, 6, 1, 2, 3, 7):
    print(f"  {names[k]:<13} {st[k] / max(1, tot) * 100:6.2f} %")
