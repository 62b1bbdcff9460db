#!/usr/bin/env python3
"""Contract drift: how far the shipped arithmetic contract (what the HIP kernels
implement bit for bit) sits from the reference's GLSL read literally.

The oracle renders the same pixels three ways (oracle/rt_oracle.cpp LIT_*):
  contract  the shipped contract (fma dot, D = fma(b, b, -a c), roots times 1/a, fma hit point)
  rint      shader.rint:33-55 as written: D = b*b - a*c, roots / a, hit point o + t*d
  all       also every dot() unfused left to right and normalize(v) = v / length(v)
and reports, for contract vs each literal form: the fraction of bit-identical accumulator
texels, of identical rgba8 pixels, and the PSNR of the rgba8 image.

Workloads: (1) blocks of the BASELINE config 3 frame (1920x1080, 10 000 spp, the bench's pixels)
in both streams: the counter-based stream and the reference's per-pixel LCG stream at the
identical seed (the north star's "PSNR >= 50 dB vs reference at identical seed"), (2) a 320x180
frame at 64 spp in both streams. `noise_floor` compares the two streams' contract renders: two
independent Monte-Carlo estimates of the same pixels, the PSNR a fully decorrelated stream reaches.
Usage: python scripts/contract_drift.py [--blocks 8 --rows 8 --width 24] [--threads N] [--out F]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from oracle import oracle  # noqa: E402  (test / measurement infrastructure)


def compare(a_acc, a_px, b_acc, b_px) -> dict:
    same_acc = np.all(a_acc[..., :3] == b_acc[..., :3], axis=-1)
    same_px = np.all(a_px[..., :3] == b_px[..., :3], axis=-1)
    mse = float(np.mean((a_px[..., :3].astype(np.float64) - b_px[..., :3]) ** 2))
    rel = np.abs(a_acc[..., :3].astype(np.float64) - b_acc[..., :3]) / np.maximum(1e-30, np.abs(b_acc[..., :3]))
    mean_a, mean_b = float(a_acc[..., :3].astype(np.float64).mean()), float(b_acc[..., :3].astype(np.float64).mean())
    return {"texels": int(same_acc.size), "accum_bit_identical": round(float(same_acc.mean()), 6),
            "image_mean_rel_diff": (mean_a - mean_b) / mean_b,
            "rgba8_identical": round(float(same_px.mean()), 6),
            "psnr_db": "inf" if mse == 0 else round(10 * np.log10(255 ** 2 / mse), 2),
            "accum_max_rel_diff": float(rel.max())}


def render3(sc, rci, w, h, rows, rng, threads):
    out = {}
    for name, lit in (("contract", oracle.LIT_CONTRACT), ("rint", oracle.LIT_RINT), ("all", oracle.LIT_ALL)):
        t0 = time.perf_counter()
        acc, px, st = oracle.render(sc, rci, w, h, rows=rows, opts=oracle.options(rng_mode=rng, lit=lit),
                                    threads=threads)
        out[name] = (acc, px, st, time.perf_counter() - t0)
    return out


def sweep(args, sc) -> int:
    """PSNR of the reference stream (identical seed) against the GLSL read literally, per spp: where
    the north star's 50-dB bar starts to hold."""
    W, H = 1920, 1080
    rows_per_block = args.rows
    ys = np.linspace(0, H - rows_per_block, args.blocks).round().astype(int)
    out = {"what": "config 3 blocks (1920x1080 frame, canonical scene), reference per-pixel LCG stream at the "
                   "reference's seed: the contract (= the kernel, bit for bit) against shader.rint:46-55 as written "
                   "(rint) and every dot / normalize as written too (all)", "rows": {}}
    for spp in [int(v) for v in args.sweep.split(",")]:
        px = int(min(W * rows_per_block * args.blocks, max(1536, args.budget / spp)))
        bw = max(1, min(W, px // (args.blocks * rows_per_block)))
        xs = np.linspace(0, W - bw, args.blocks).round().astype(int)[::-1]
        parts = {k: [] for k in ("contract", "rint", "all")}
        t0 = time.perf_counter()
        for y, x in zip(ys, xs):
            rows = np.arange(y, y + rows_per_block, dtype=np.uint32)
            r = render3(sc, oracle.render_call_info(spp, W, H, (int(x), 0)), bw, rows_per_block, rows, 0, args.threads)
            for k in parts:
                parts[k].append(r[k][:2])
        cat = {k: (np.concatenate([p[0] for p in v]), np.concatenate([p[1] for p in v])) for k, v in parts.items()}
        out["rows"][spp] = {"pixels": int(args.blocks * rows_per_block * bw),
                            "blocks": f"{args.blocks} blocks of {rows_per_block} rows x {bw} px",
                            "rint_literal": compare(*cat["rint"], *cat["contract"]),
                            "all_literal": compare(*cat["all"], *cat["contract"]),
                            "cpu_s": round(time.perf_counter() - t0, 1)}
        print(f"{spp} spp: {out['rows'][spp]['pixels']} px, rint {out['rows'][spp]['rint_literal']['psnr_db']} dB, "
              f"all {out['rows'][spp]['all_literal']['psnr_db']} dB", flush=True)
    print(json.dumps(out, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--rows", type=int, default=8)
    ap.add_argument("--width", type=int, default=24)
    ap.add_argument("--spp", type=int, default=10000)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=None, help="also write the JSON here")
    ap.add_argument("--sweep", default=None,
                    help="spp list (e.g. 64,256,1000,10000): the reference stream at the identical seed against "
                         "both literal forms on config 3's blocks at each spp, the block width scaled so every spp "
                         "renders about --budget samples per form")
    ap.add_argument("--budget", type=float, default=2.4e7)
    args = ap.parse_args()
    oracle.build()
    sc = oracle.generate_scene(0.0)
    if args.sweep:
        return sweep(args, sc)
    res = {}
    # (1) config 3 blocks, counter-based stream (the bench's stream), spread like bench.py's cpu_baseline
    W, H = 1920, 1080
    ys = np.linspace(0, H - args.rows, args.blocks).round().astype(int)
    xs = np.linspace(0, W - args.width, args.blocks).round().astype(int)[::-1]
    cat_by_stream = {}
    for rng, sname in ((2, "hash"), (0, "stream")):
        parts = {k: [] for k in ("contract", "rint", "all")}
        secs = 0.0
        for y, x in zip(ys, xs):
            rows = np.arange(y, y + args.rows, dtype=np.uint32)
            r = render3(sc, oracle.render_call_info(args.spp, W, H, (int(x), 0)), args.width, args.rows, rows,
                        rng, args.threads)
            for k in parts:
                parts[k].append(r[k][:2])
            secs += sum(v[3] for v in r.values())
        cat = {k: (np.concatenate([p[0] for p in v]), np.concatenate([p[1] for p in v])) for k, v in parts.items()}
        cat_by_stream[sname] = cat
        res["config3_blocks" if sname == "hash" else "config3_blocks_reference_stream"] = {
            "pixels": f"{args.blocks} blocks of {args.rows} rows x {args.width} px of 1920x1080 at {args.spp} spp, "
                      + ("hash stream" if sname == "hash" else "reference per-pixel LCG stream (identical seed)"),
            "rint_literal": compare(*cat["rint"], *cat["contract"]),
            "all_literal": compare(*cat["all"], *cat["contract"]),
            "cpu_s": round(secs, 1)}
    res["config3_blocks_noise_floor"] = {
        "what": "contract render, reference stream vs hash stream: two independent estimates of the same pixels",
        **compare(*cat_by_stream["stream"]["contract"], *cat_by_stream["hash"]["contract"])}
    # (2) 320x180 at 64 spp, both streams
    for rng, name in ((0, "stream"), (2, "hash")):
        r = render3(sc, oracle.render_call_info(64, 320, 180), 320, 180, None, rng, args.threads)
        res[f"320x180_64spp_{name}"] = {
            "rint_literal": compare(*r["rint"][:2], *r["contract"][:2]),
            "all_literal": compare(*r["all"][:2], *r["contract"][:2]),
            "segments": {k: v[2][0] for k, v in r.items()}}
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
