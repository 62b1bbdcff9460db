"""Config 4 on one GPU: each rank's band of the N-GPU frame (rows = rtvk.dist.strip_rows(r, N, H)),
rendered alone at the shipped build, in the counter-based stream. For every rank: the trace
kernel's duration (HIP events the library records on the launch stream, rt_debug_kernel_times)
after a warm-up launch of the same band (the LPT order of that band geometry), and the sample
chunks per pixel the library picked. Reports the predicted N-GPU frame (the slowest band), the
imbalance (max / mean) and the efficiency against the one-GPU frame timed the same way.

usage: python scripts/band_probe.py [N=8] [spp=10000] [--ranks 0,1,...] [--reps 2] [--json out]
The PMC WRITE_SIZE of one band comes from running this under rocprofv3 with --ranks r."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))
import torch  # noqa: E402

import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402
from rtvk.dist import strip_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="?", default=8)
ap.add_argument("spp", type=int, nargs="?", default=10000)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--ranks", default=None)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--no-full", action="store_true", help="skip the one-GPU frame")
ap.add_argument("--json", default=None)
args = ap.parse_args()
W, H, N = args.width, args.height, args.n
ranks = [int(x) for x in args.ranks.split(",")] if args.ranks else list(range(N))
r = rtvk.Renderer(0)
r.set_scene(rtvk.generateRandomScene())
rci = rtvk.canonical_render_call_info(args.spp, W, H)
opt = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=rtvk.HASH)


def timed(rows_np):
    n = H if rows_np is None else len(rows_np)
    rows = None if rows_np is None else torch.from_numpy(rows_np).cuda()
    acc = torch.zeros((n, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((n, W, 4), dtype=torch.uint8, device="cuda")
    r.render_device(rci, acc, out, rows=rows, options=opt)   # warm-up: LPT order of this band geometry
    torch.cuda.synchronize()
    for _ in range(args.reps):
        r.render_device(rci, acc, out, rows=rows, options=opt)
    torch.cuda.synchronize()
    ks = r.kernel_times(args.reps)
    info = r.launch_info()
    return sum(ks) / len(ks), info


res = {"n": N, "width": W, "height": H, "spp": args.spp, "lib": abi.build_info().get("sources_sha256"),
       "ranks": {}}
t0 = time.perf_counter()
for rk in ranks:
    rows = strip_rows(rk, N, H)
    ms, info = timed(rows)
    res["ranks"][rk] = {"rows": int(len(rows)), "kernel_ms": round(ms, 3), "chunks": info["chunks"],
                        "head_chunks": info["head_chunks"]}
    print(f"rank {rk}: {len(rows)} rows, {ms:.2f} ms, chunks {info['chunks']} (head {info['head_chunks']})",
          flush=True)
ks = [v["kernel_ms"] for v in res["ranks"].values()]
res["max_ms"] = max(ks)
res["mean_ms"] = round(sum(ks) / len(ks), 3)
res["imbalance"] = round(max(ks) / (sum(ks) / len(ks)), 4)
if not args.no_full:
    full_ms, finfo = timed(None)
    res["one_gpu_ms"] = round(full_ms, 3)
    res["one_gpu_chunks"] = finfo["chunks"]
    if len(ranks) == N:
        res["predicted_efficiency"] = round(full_ms / (N * max(ks)), 4)
        res["predicted_msamples_per_s"] = round(W * H * args.spp / (max(ks) * 1e-3) / 1e6, 1)
res["seconds"] = round(time.perf_counter() - t0, 1)
print(json.dumps(res), flush=True)
if args.json:
    Path(args.json).write_text(json.dumps(res, indent=1))
r.close()
