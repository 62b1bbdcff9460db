"""Configs 4 and 5 on one GPU: each rank's band of the N-GPU frame rendered alone at the shipped
build, in the counter-based stream, one context per rank (as each GPU has its own), and the
cross-device balancer iterated on the measured band times.

Iteration 0 is the row-exact strips (rtvk.partition_strips, the partition every multi-GPU frame
starts from). After each iteration every rank's band time (the trace kernel, HIP events the
library records on the launch stream) and per-row work (its tile-cost record,
rt_launch_row_weights) become per-row cost estimates (rtvk.dist.row_costs) and the partition is
re-dealt (rtvk.partition_rebalance) — what rt_multi and rtvk.dist do between frames with a lag of
two frames. Each band is rendered once before it is timed (its LPT order; after a re-deal the
context's record is carried over, as on the real devices). With --rebuild every render is preceded
by the per-frame scene rebuild (config 5: the device LBVH + grid build of all spheres, which every
rank repeats per frame), and the step (rebuild + render, synchronised) is timed too.

Reports per iteration the rows, kernel ms and sample chunks of every rank, the imbalance (max /
mean) and the predicted efficiency against the one-GPU frame timed the same way.

usage: python scripts/band_probe.py [N=8] [spp=10000] [--width W --height H --grid K] [--iters 4]
       [--ranks 0,1,...] [--reps 2] [--rebuild] [--no-full] [--json out]
The PMC WRITE_SIZE of one band comes from running this under rocprofv3 with --ranks r --iters 0."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402
from rtvk.dist import blend_costs, row_costs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="?", default=8)
ap.add_argument("spp", type=int, nargs="?", default=10000)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--grid", type=int, default=11)
ap.add_argument("--iters", type=int, default=4, help="balancer re-deals after the row-exact strips")
ap.add_argument("--ranks", default=None)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--rebuild", action="store_true", help="rebuild the scene before every render (per-frame build)")
ap.add_argument("--no-full", action="store_true", help="skip the one-GPU frame")
ap.add_argument("--json", default=None)
args = ap.parse_args()
W, H, N = args.width, args.height, args.n
ranks = [int(x) for x in args.ranks.split(",")] if args.ranks else list(range(N))
scene = rtvk.generateRandomScene(0.0, args.grid)
ctxs = {}
rci = rtvk.canonical_render_call_info(args.spp, W, H)
opt = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=rtvk.HASH)


def ctx(key):
    if key not in ctxs:
        r = rtvk.Renderer(0)
        r.set_scene(scene)
        try:   # the first call switches the context's tile-cost record copies on (finds none)
            r.launch_row_weights(1, 0)
        except rtvk.RtError:
            pass
        ctxs[key] = r
    return ctxs[key]


def timed(key, rows_np):
    r = ctx(key)
    n = H if rows_np is None else len(rows_np)
    rows = None if rows_np is None else torch.from_numpy(np.asarray(rows_np, np.int32)).cuda()
    acc = torch.zeros((n, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((n, W, 4), dtype=torch.uint8, device="cuda")
    if args.rebuild:
        r.set_scene(scene)
    r.render_device(rci, acc, out, rows=rows, options=opt)   # warm-up: LPT order of this band geometry
    torch.cuda.synchronize()
    steps = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        if args.rebuild:
            r.set_scene(scene)
        r.render_device(rci, acc, out, rows=rows, options=opt)
        torch.cuda.synchronize()
        steps.append((time.perf_counter() - t0) * 1e3)
    ks = r.kernel_times(args.reps)
    info = r.launch_info()
    w = r.launch_row_weights(n, 0)
    return sum(ks) / len(ks), sum(steps) / len(steps), info, w


res = {"n": N, "width": W, "height": H, "spp": args.spp, "spheres": len(scene), "rebuild": args.rebuild,
       "lib": abi.build_info().get("sources_sha256"), "iterations": []}
t0 = time.perf_counter()
full_ms = None
if not args.no_full:
    full_ms, full_step, finfo, _ = timed("full", None)
    res["one_gpu_ms"] = round(full_ms, 3)
    res["one_gpu_step_ms"] = round(full_step, 3)
    res["one_gpu_chunks"] = finfo["chunks"]
    print(f"one GPU: {full_ms:.2f} ms kernel, {full_step:.2f} ms step", flush=True)
parts = rtvk.partition_strips(N, H)
cost = np.zeros(H, np.float64)
for it in range(args.iters + 1):
    row = {"rows": [], "kernel_ms": [], "step_ms": [], "chunks": []}
    new = np.zeros(H, np.float64)
    for rk in ranks:
        ms, step, info, w = timed(rk, parts[rk])
        row["rows"].append(int(len(parts[rk])))
        row["kernel_ms"].append(round(ms, 3))
        row["step_ms"].append(round(step, 3))
        row["chunks"].append([info["chunks"], info["head_chunks"]])
        new[parts[rk]] = row_costs(parts[rk], ms, w)
    cost = blend_costs(cost, new, 0.5)   # as rtvk.dist / rt_multi between frames
    ks = row["kernel_ms"]
    row["max_ms"] = max(ks)
    row["mean_ms"] = round(sum(ks) / len(ks), 3)
    row["imbalance"] = round(max(ks) / (sum(ks) / len(ks)), 5)
    if full_ms and len(ranks) == N:
        row["predicted_efficiency"] = round(full_ms / (N * max(ks)), 4)
        row["predicted_msamples_per_s"] = round(W * H * args.spp / (max(ks) * 1e-3) / 1e6, 1)
        row["predicted_step_efficiency"] = round(res["one_gpu_step_ms"] / (N * max(row["step_ms"])), 4)
    print(f"iteration {it}: rows {row['rows']}, kernel ms {ks}, imbalance {row['imbalance']}, "
          f"efficiency {row.get('predicted_efficiency')}", flush=True)
    res["iterations"].append(row)
    if it < args.iters and len(ranks) == N:
        parts, moved, pred = rtvk.partition_rebalance(parts, cost)
        row["rows_moved_after"] = moved
        row["predicted_imbalance_after"] = round(pred, 5)
        if not moved:
            break
res["first"] = {k: res["iterations"][0].get(k) for k in ("imbalance", "predicted_efficiency", "rows")}
res["last"] = {k: res["iterations"][-1].get(k) for k in ("imbalance", "predicted_efficiency", "rows")}
res["seconds"] = round(time.perf_counter() - t0, 1)
print(json.dumps(res), flush=True)
if args.json:
    Path(args.json).write_text(json.dumps(res, indent=1))
for r in ctxs.values():
    r.close()
