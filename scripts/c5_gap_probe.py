#!/usr/bin/env python3
"""Per-frame overhead of the device-built scene path (config 5 shape: 4K, 99 860 spheres, a device
LBVH + grid build every frame): step time minus trace-kernel time, and where the host waits.

For each library (the default build, then any variants given), frames are issued as bench.py
issues them — rt_set_scene then rt_render_device on one stream — and per frame the host records
how long rt_set_scene blocked (it waits for the build's summary) and how long rt_render_device
took to return. The multi path (rt_multi at one GPU) runs too. Rounds are interleaved so drift
hits every library alike; every library's image must equal the default's.

--solo PATH LIB: one library and one path in this process, with bench.py's streams (single: a
stream of its own for set_scene and render; multi: torch's current stream as the caller's), so
the hardware-queue assignment of the streams is the bench's (it depends on what else the process
created: the shared form above mixes several contexts' streams).

usage: python scripts/c5_gap_probe.py [--spp 100] [--frames 8] [--rounds 2] [variant.so ...]
       python scripts/c5_gap_probe.py --solo single|multi lib.so [--spp 1000] [--frames 5]
"""
import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))

import torch  # noqa: E402

import rtvk  # noqa: E402
from rtvk import abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--grid", type=int, default=158)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--no-multi", action="store_true")
    ap.add_argument("--solo", choices=["single", "multi"])
    args = ap.parse_args()
    if args.solo and len(args.libs) != 1:
        ap.error("--solo takes exactly one library")
    W, H = args.width, args.height
    scene = rtvk.generateRandomScene(0.0, args.grid)
    rci = rtvk.canonical_render_call_info(args.spp, W, H)
    opt = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=abi.RT_RNG_SAMPLE_HASH)
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev) if args.solo != "multi" else None
    sp = stream.cuda_stream if stream is not None else None
    libs = [str(abi.LIB_PATH)] + args.libs
    if args.solo:
        libs = args.libs
        if args.solo == "multi":
            sp = torch.cuda.current_stream(dev).cuda_stream
    runs = []
    for lp in libs:
        if args.solo == "multi":
            break
        lib = abi.load_library(lp)
        ctx = ctypes.c_void_p()
        assert lib.rt_context_create(0, ctypes.byref(ctx)) == 0, lib.rt_last_error()
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
        runs.append({"lib": Path(lp).name, "L": lib, "ctx": ctx, "acc": acc, "out": out})
    bases = runs[:] if not args.solo else [{"lib": Path(libs[0]).name, "L": abi.load_library(libs[0])}]
    for r in bases:
        if args.no_multi or args.solo == "single":
            break
        m = ctypes.c_void_p()
        assert r["L"].rt_multi_create(1, ctypes.byref(m)) == 0, r["L"].rt_last_error()
        runs.append({"lib": "multi:" + r["lib"], "L": r["L"], "m": m,
                     "acc": torch.zeros((H, W, 4), dtype=torch.float32, device=dev),
                     "out": torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)})

    def frame(r, t):
        L = r["L"]
        t0 = time.perf_counter()
        if "m" in r:
            assert L.rt_multi_set_scene(r["m"], ctypes.addressof(scene), len(scene)) == 0, L.rt_last_error()
        else:
            assert L.rt_set_scene(r["ctx"], ctypes.addressof(scene), len(scene), sp) == 0, L.rt_last_error()
        t1 = time.perf_counter()
        if "m" in r:
            assert L.rt_multi_render(r["m"], ctypes.byref(rci), ctypes.byref(opt), r["acc"].data_ptr(),
                                     r["out"].data_ptr(), sp) == 0, L.rt_last_error()
        else:
            assert L.rt_render_device(r["ctx"], ctypes.byref(rci), None, W, H, r["acc"].data_ptr(),
                                      r["out"].data_ptr(), ctypes.byref(opt), sp) == 0, L.rt_last_error()
        t2 = time.perf_counter()
        t["scene"].append((t1 - t0) * 1e3)
        t["render"].append((t2 - t1) * 1e3)

    def kernel_ms(r, n):
        L = r["L"]
        got = ctypes.c_uint32()
        if "m" in r:
            buf = (ctypes.c_float * n)()
            assert L.rt_multi_kernel_times_frames(r["m"], n, buf, n, ctypes.byref(got)) == 0
        else:
            buf = (ctypes.c_float * n)()
            assert L.rt_debug_kernel_times(r["ctx"], buf, n, ctypes.byref(got)) == 0
        return list(buf[: got.value])

    results = {}
    for rnd in range(args.rounds):
        for r in runs:
            name = r["lib"]
            t = {"scene": [], "render": []}
            for _ in range(2):   # warm: LPT history, both arenas, occupancy
                frame(r, t)
            torch.cuda.synchronize(dev)
            t["scene"].clear()
            t["render"].clear()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                frame(r, t)
            torch.cuda.synchronize(dev)
            el = (time.perf_counter() - t0) * 1e3 / args.frames
            ks = kernel_ms(r, args.frames)
            km = sum(ks) / max(1, len(ks))
            rec = {"round": rnd, "ms_per_step": round(el, 4), "kernel_ms": round(km, 4),
                   "overhead_ms": round(el - km, 4),
                   "set_scene_host_ms": [round(x, 2) for x in t["scene"]],
                   "render_host_ms": [round(x, 2) for x in t["render"]]}
            results.setdefault(name, []).append(rec)
            print(json.dumps({"lib": name, **rec}), flush=True)
    ref = runs[0]["out"].cpu()
    for r in runs[1:]:
        if not torch.equal(ref, r["out"].cpu()):
            print(json.dumps({"lib": r["lib"], "image": "DIFFERS from the default build"}), flush=True)
            return 1
    summary = {k: round(sum(x["overhead_ms"] for x in v) / len(v), 4) for k, v in results.items()}
    print(json.dumps({"mean_overhead_ms": summary, "spp": args.spp, "frames": args.frames}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
