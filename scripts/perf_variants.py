#!/usr/bin/env python3
"""A/B timing of librt_mi355x.so build variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24). Every variant must produce the default build's image
bit-exactly. Usage: python scripts/perf_variants.py [--spp 100] [--rounds 3] lib1.so lib2.so ..."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--accels", default="2,1")
    ap.add_argument("--walk", default="0", help="LBVH walk forms to sweep (0 default/ordered, 1 escape-link)")
    ap.add_argument("--count", action="store_true", help="also report box / sphere tests per segment")
    ap.add_argument("--rng", default="0", help="rng modes to sweep (0 pixel stream, 1 sample counter)")
    ap.add_argument("--inexact", action="store_true",
                    help="report differing pixels instead of failing (experiments that relax exactness)")
    args = ap.parse_args()
    libs = [str(abi.LIB_PATH)] + args.libs
    W, H = args.width, args.height
    scene = rtvk.generateRandomScene(0.0, args.grid)
    rci = rtvk.canonical_render_call_info(args.spp, W, H)
    stream = torch.cuda.current_stream()
    ctxs = []
    for lp in libs:
        lib = abi.load_library(lp)
        ctx = ctypes.c_void_p()
        assert lib.rt_context_create(0, ctypes.byref(ctx)) == 0, lib.rt_last_error()
        assert lib.rt_set_scene(ctx, ctypes.addressof(scene), len(scene), None) == 0
        ctxs.append((lp, lib, ctx))
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    times = {}
    stamps = {}
    ref = {}
    configs = []
    for accel in [int(a) for a in args.accels.split(",")]:
        for c in ([int(x) for x in args.walk.split(",")] if accel == 2 else [0]):
            for rng in [int(x) for x in args.rng.split(",")]:
                opt = rtvk.make_options(accel=accel, rng_mode=rng)
                opt.reserved[1] = c
                configs.append((accel * 10 + rng, c, opt))
    for accel, cth, opt in configs:
        for r in range(args.rounds + 1):
            for lp, lib, ctx in ctxs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rc = lib.rt_render_device(ctx, ctypes.byref(rci), None, W, H, acc.data_ptr(), out.data_ptr(),
                                          ctypes.byref(opt), stream.cuda_stream)
                e1.record(stream)
                assert rc == 0, lib.rt_last_error()
                torch.cuda.synchronize()
                if r == 0 and args.count:
                    copt = rtvk.make_options(accel=accel // 10, count_tests=True, rng_mode=accel % 10)
                    copt.reserved[1] = cth
                    assert lib.rt_render_device(ctx, ctypes.byref(rci), None, W, H, acc.data_ptr(), out.data_ptr(),
                                                ctypes.byref(copt), stream.cuda_stream) == 0
                    torch.cuda.synchronize()
                    cs = rtvk.Stats()
                    assert lib.rt_get_stats(ctx, ctypes.byref(cs)) == 0
                    u32 = (ctypes.c_uint64 * 32)()
                    fb = int(u32[30]) if hasattr(lib, "rt_debug_util") and lib.rt_debug_util(ctx, u32) == 0 else None
                    print(json.dumps({"lib": Path(lp).name, "accel": accel, "walk": cth,
                                      "box_per_seg": round(cs.box_tests / max(1, cs.segments), 3),
                                      "sphere_per_seg": round(cs.sphere_tests / max(1, cs.segments), 3),
                                      "segments": int(cs.segments), "gate_fallbacks": fb}), flush=True)
                if r == 0:  # warm-up round doubles as the bit-exactness check
                    img = acc.cpu().numpy()
                    if accel not in ref:
                        ref[accel] = img
                    if args.inexact:
                        bad = int(np.any(img != ref[accel], axis=-1).sum())
                        print(json.dumps({"lib": Path(lp).name, "accel": accel, "pixels_differing": bad}))
                    else:
                        assert np.array_equal(img, ref[accel]), f"{lp} differs from the default build"
                    continue
                times.setdefault((accel, cth, Path(lp).name), []).append(e0.elapsed_time(e1))
                st8 = (ctypes.c_uint64 * 8)()
                if lib.rt_debug_stamps(ctx, st8) == 0 and any(st8):
                    tot = sum(st8)
                    stamps.setdefault((accel, cth, Path(lp).name), [round(v / tot, 4) for v in st8])
    rows = []
    for (accel, cth, name), ts in sorted(times.items()):
        ms = float(np.median(ts))
        rows.append({"accel": accel, "walk": cth, "lib": name, "ms_median": round(ms, 3), "ms_min": round(min(ts), 3),
                     "msamples_s": round(W * H * args.spp / ms / 1e3, 1)})
    for r in rows:
        print(json.dumps(r))
    for k, v in stamps.items():
        print(json.dumps({"stamps": list(k), "share": v}))


if __name__ == "__main__":
    main()
