"""Diagnostic: per-segment latency of one wave running alone. Renders a tiny image (one 8x8 tile
per wave, a handful of waves on an idle GPU) and divides the launch time by its longest pixel
chain (segments of the most expensive pixel, recorded for the LPT hand-out)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import torch  # noqa: E402
import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402

lib = abi.load_library()
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
for W, H, spp in [(8, 8, 100), (32, 32, 100), (64, 64, 100), (256, 256, 100)]:
    rci = rtvk.canonical_render_call_info(spp, W, H)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    ts = []
    for i in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render_device(rci, acc, out, options=rtvk.make_options(accel=2))
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    n = ctypes.c_uint64()
    abi.check(lib.rt_debug_tile_cost(r._ctx, None, 0, ctypes.byref(n)))
    c = (ctypes.c_uint32 * n.value)()
    abi.check(lib.rt_debug_tile_cost(r._ctx, c, n.value, ctypes.byref(n)))
    c = np.array(c, np.float64)
    ms = float(np.median(ts))
    st = r.stats()
    print(f"{W}x{H} @ {spp} spp: {ms:.2f} ms, {int(n.value)} tiles, longest chain {c.max():.0f} segments, "
          f"mean pixel {st.segments / (W * H):.0f} -> {ms * 1e3 / c.max():.2f} us per segment of the longest chain",
          flush=True)
