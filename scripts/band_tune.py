"""A/B of the launch plan (rt_debug_tune) on one rank's band of the N-GPU frame (config 4's band
geometry, rows = rtvk.dist.strip_rows(rank, N, H)), in one process, interleaved rounds: the trace
kernel's duration (HIP events on the launch stream) and the tail after the work queue ran dry
(s_memrealtime stamps of the launch, rt_debug_lane_hist), per setting. Every setting renders the
same image (checked against the first setting's, bit for bit).

usage: python scripts/band_tune.py [N=8] [spp=10000] [--rank 0] [--rounds 3] [--full]
       [--width W --height H --grid K] [--rng hash|stream] [--set name:key=v,key=v ...]
       (default sets below)"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402


DEFAULT_SETS = [
    "default:",
    "min128:unit_min_samples=128",
    "min64:unit_min_samples=64",
    "head10:head_chunks=10",
    "head39:head_chunks=39",
    "tail300:tail_tiles_pm=300",
    "min128_tail300:unit_min_samples=128,tail_tiles_pm=300",
]

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="?", default=8)
ap.add_argument("spp", type=int, nargs="?", default=10000)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--full", action="store_true", help="the whole frame instead of one band")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--grid", type=int, default=11)
ap.add_argument("--rng", choices=["hash", "stream"], default="hash")
ap.add_argument("--set", nargs="*", default=None)
args = ap.parse_args()
W, H = args.width, args.height
sets = []
for spec in (args.set or DEFAULT_SETS):
    name, _, kv = spec.partition(":")
    d = {}
    for item in filter(None, kv.split(",")):
        k, v = item.split("=")
        d[k] = float(v)
    sets.append((name, d))
lib = abi.load_library()
scene = rtvk.generateRandomScene(0.0, args.grid)
rci = rtvk.canonical_render_call_info(args.spp, W, H)
opt = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=rtvk.HASH if args.rng == "hash" else rtvk.STREAM)
rows_np = None if args.full else rtvk.partition_strips(args.n, H)[args.rank].astype(np.int32)
n = H if rows_np is None else len(rows_np)
rows = None if rows_np is None else torch.from_numpy(rows_np).cuda()
ctxs = []
for name, kv in sets:   # one context per setting: its own LPT history for this geometry
    r = rtvk.Renderer(0)
    r.set_scene(scene)
    r.tune(**kv)
    a = torch.zeros((n, W, 4), dtype=torch.float32, device="cuda")
    o = torch.zeros((n, W, 4), dtype=torch.uint8, device="cuda")
    r.render_device(rci, a, o, rows=rows, options=opt)   # warm: LPT order
    ctxs.append((name, r, a, o))
torch.cuda.synchronize()
res = {name: {"ms": [], "tail_ms": [], "chunks": None} for name, _ in sets}
ref = None
for rd in range(args.rounds):
    for name, r, a, o in ctxs:
        r.render_device(rci, a, o, rows=rows, options=opt)
        torch.cuda.synchronize()
        res[name]["ms"].append(r.kernel_times(1)[0])
        h = (ctypes.c_uint64 * 68)()
        abi.check(lib.rt_debug_lane_hist(r._ctx, h))
        res[name]["tail_ms"].append((h[67] - h[66]) / 1e5)
        info = r.launch_info()
        res[name]["chunks"] = [info["head_chunks"], info["chunks"]]
        img = a.cpu().numpy()
        if ref is None:
            ref = img
        assert np.array_equal(img, ref), f"{name}: image differs"
base = float(np.median(res[sets[0][0]]["ms"]))
for name, v in res.items():
    ms = float(np.median(v["ms"]))
    print(f"{name:18s} {ms:9.2f} ms ({(ms / base - 1) * 100:+5.1f} %)  tail after queue dry "
          f"{np.median(v['tail_ms']):6.2f} ms  chunks head/tail {v['chunks']}", flush=True)
print(json.dumps({"n": args.n, "rank": args.rank, "spp": args.spp, "rng": args.rng, "full": args.full, "rows": n, "results": res}))
