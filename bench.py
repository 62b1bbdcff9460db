#!/usr/bin/env python3
"""bench.py — Msamples/s of the MI355X path tracer on the canonical RTIOW scene (BASELINE.json).

One step = one frame of the hot path: every pixel of the 1920x1080 image traced at `--spp`
samples, depth 50, on the canonical scene (generateRandomScene(t=0): 488 spheres, camera
(13,11,-3) -> origin), i.e. BASELINE.json config 2's input. For N > 1 the step also includes the
RCCL gather of every rank's row strips to rank 0 and the on-device reassembly (strong scaling:
the image is fixed, each GPU renders 1/N of its rows).

Launch: python bench.py [--gpus 1 --steps 5 --warmup 2]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Rank 0 prints one JSON line (DESIGN.md §6 explains every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))

VALU_FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, vector FP32 (256 CU x 2.4 GHz)
HBM_PEAK_GBPS = 8000.0
FLOP_PER_SPHERE_TEST = 23
FLOP_PER_BOX_TEST = 20
BYTES_PER_BOX_TEST = 32         # bytes/sample = S·(B·32 + T·16), read from LDS
BYTES_PER_SPHERE_TEST = 16
LDS_PEAK_TBPS = 256 * 256 * 2.4e9 / 1e12   # ds_read_b128: 256 B/clk/CU (MI355X_MICROARCH.md §LDS) x 256 CU x 2.4 GHz


def host_cores() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))    # the GPU box grants a 16-CPU share


def cpu_baseline(width: int, height: int, spp: int, gpu_accum=None, gpu_rgba8=None,
                 target_s: float = 15.0) -> dict:
    """The CPU oracle (C++ restatement of the shaders, brute-force closest hit) on this host's
    cores, on a bounded sample of the bench workload itself: evenly spaced rows of the bench frame
    at its full spp, sized to ~`target_s` of CPU work from a timed config-1 frame (1920x1080 at
    1 spp). Msamples/s is spp-independent. The same rows of the GPU's bench frame
    (gpu_accum / gpu_rgba8, numpy [H, W, 4]) are compared with the oracle's: exact match and PSNR
    of the rgba8 image (BASELINE.json's "PSNR vs CPU ref")."""
    import numpy as np
    from oracle import oracle
    oracle.build()
    sc = oracle.generate_scene(0.0)
    threads = host_cores()
    t0 = time.perf_counter()
    _, _, st1 = oracle.render(sc, oracle.render_call_info(1, width, height), width, height, threads=threads)
    t1 = time.perf_counter() - t0
    per_row = t1 / height * spp   # seconds per row of the bench frame
    if per_row * threads > target_s:   # one row per thread would already exceed the budget
        return {"value": round(width * height / t1 / 1e6, 4), "unit": "Msamples/s", "cores": threads,
                "kind": "port",
                "sample": f"config 1 frame ({width}x{height}, 1 spp, depth 50), brute-force closest hit, "
                          f"{threads} threads, {t1:.2f} s (rows of the {spp}-spp bench frame would exceed "
                          f"{target_s:.0f} s)", "config1_frame_s": round(t1, 3)}
    n_rows = int(max(threads, min(height, round(target_s / max(per_row, 1e-9)))))
    rows = np.unique(np.linspace(0, height - 1, n_rows).round().astype(np.uint32))
    t0 = time.perf_counter()
    acc, out, st = oracle.render(sc, oracle.render_call_info(spp, width, height), width, len(rows),
                                 rows=rows, threads=threads)
    dt = time.perf_counter() - t0
    res = {"value": round(width * len(rows) * spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
           "kind": "port",
           "sample": f"{len(rows)} evenly spaced rows of the bench frame ({width} px, {spp} spp, depth 50), "
                     f"brute-force closest hit, {threads} threads, {dt:.2f} s; config 1 frame "
                     f"({width}x{height}, 1 spp) alone {t1:.2f} s; {st[0] / max(1, st[1]):.3f} segments/sample",
           "config1_frame_s": round(t1, 3)}
    if gpu_accum is not None and gpu_rgba8 is not None:
        ga, go = gpu_accum[rows.astype(np.int64)], gpu_rgba8[rows.astype(np.int64)]
        mse = float(np.mean((go[..., :3].astype(np.float64) - out[..., :3].astype(np.float64)) ** 2))
        res["parity"] = {"rows": int(len(rows)), "accum_bit_exact": bool(np.array_equal(ga, acc)),
                         "rgba8_equal": bool(np.array_equal(go, out)),
                         "psnr_db": "inf" if mse == 0.0 else round(float(10.0 * np.log10(255.0 ** 2 / mse)), 2)}
    return res


def _pmc_record(path: Path, key: str):
    """A committed rocprofv3 --pmc summary (scripts/pmc_to_json.py) for this workload, or None."""
    try:
        return json.loads(path.read_text()).get(key)
    except (OSError, ValueError):
        return None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--accel", choices=["lbvh", "brute"], default="lbvh")
    ap.add_argument("--grid", type=int, default=11, help="scene grid half extent (11: 488 spheres)")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=None,
                    help="BASELINE.json config preset: 2/3/4 = 1920x1080 at 100/10000/10000 spp, "
                         "5 = 3840x2160, 99 860 spheres, 1000 spp (overrides --width/--height/--spp/--grid)")
    ap.add_argument("--count-spp", type=int, default=100,
                    help="spp of the instrumented (test-counting) launch; its counts are scaled to --spp "
                         "(per-sample statistics are stationary: same scene, same per-pixel streams)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-brute-line", action="store_true", help="skip the brute-force side measurement")
    ap.add_argument("--profile", action="store_true", help="short run for rocprofv3 (no side legs)")
    ap.add_argument("--walk", type=int, default=0,
                    help="LBVH walk form (A/B only): 0 default escape-link, 2 ordered, 4 compact nodes")
    ap.add_argument("--split", choices=["samples", "strips"], default="samples",
                    help="N>1 work split: samples (each rank renders the frame with spp/N samples and "
                         "stream salt number+rank, row-slice reduction) or strips (8-row strips of the "
                         "one-GPU frame); identical at N=1")
    ap.add_argument("--inflight", type=int, default=2,
                    help="frames in flight: contexts + streams used round robin, so frame k+1's blocks "
                         "start on the CUs frame k's tail leaves idle (1 = one frame at a time)")
    ap.add_argument("--exchange-test", action="store_true",
                    help="test only: one rank on a one-rank NCCL group still runs the sample-split "
                         "exchange (RCCL code path on a one-GPU box)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import rtvk
    from rtvk import abi
    from rtvk.dist import (DistributedRenderer, SampleSplitRenderer, hip_assembler, hip_band_renderer,
                           hip_full_renderer, hip_reducer)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # RT_SHARE_DEVICE=1 (rehearsal only): map ranks onto the visible devices round robin, so the
    # multi-rank code path can be exercised on a one-GPU box.
    ndev = torch.cuda.device_count()
    # RCCL refuses two ranks on one device, so the rehearsal runs over gloo with host staging.
    shared = os.environ.get("RT_SHARE_DEVICE") == "1" and ndev > 0
    if shared:
        local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.exchange_test:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    if args.exchange_test:
        import rtvk.dist as rtvk_dist
        rtvk_dist._force_collective = True

    if args.config is not None:
        args.width, args.height = (3840, 2160) if args.config == 5 else (1920, 1080)
        args.spp = {2: 100, 3: 10000, 4: 10000, 5: 1000}[args.config]
        args.grid = 158 if args.config == 5 else 11
    W, H, spp = args.width, args.height, args.spp
    accel = abi.RT_ACCEL_BRUTE if args.accel == "brute" else abi.RT_ACCEL_LBVH
    scene = rtvk.generateRandomScene(0.0, args.grid)
    rci = rtvk.canonical_render_call_info(spp, W, H)
    opts = rtvk.make_options(accel=accel)
    opts.reserved[1] = args.walk
    ev = []
    split = args.split if (world > 1 or args.exchange_test) else "strips"

    def timed(fn):
        """fn(*a) bracketed by HIP events on the stream it is launched on (the slot's)."""
        def run(*a):
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn(*a)
            e1.record(st)
            ev.append((e0, e1))
        return run

    class Slot:
        """One frame in flight: its own context (scene blob, counters, LPT history), stream and
        frame buffers; frames go to the slots round robin."""
        def __init__(self):
            self.renderer = rtvk.Renderer(local)
            self.stream = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(self.stream):
                if split == "samples":
                    self.dr = SampleSplitRenderer(W, H, spp, rci.number, dev,
                                                  timed(hip_full_renderer(self.renderer, rci, opts)),
                                                  hip_reducer(self.renderer))
                else:
                    self.dr = DistributedRenderer(W, H, dev, timed(hip_band_renderer(self.renderer, rci, opts)),
                                                  hip_assembler(self.renderer))

        def frame(self):
            # The reference rebuilds its acceleration structure every frame (src/vulkan.h:1020-1059)
            # and SURVEY.md 8(d) counts the build in the wall clock: rebuild, then render + exchange.
            # The host build runs while earlier frames render (its upload is queued behind them).
            with torch.cuda.stream(self.stream):
                self.renderer.set_scene(scene, stream=self.stream)
                self.dr.step()

    slots = [Slot() for _ in range(max(1, args.inflight))]
    renderer, dr = slots[0].renderer, slots[0].dr
    torch.cuda.synchronize()
    t_scene = time.perf_counter()
    renderer.set_scene(scene)
    torch.cuda.synchronize()
    t_scene = time.perf_counter() - t_scene

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    n_frames = 0

    def frame():
        nonlocal n_frames
        slots[n_frames % len(slots)].frame()
        n_frames += 1

    for _ in range(max(args.warmup, len(slots))):   # every slot has rendered once (LPT order)
        frame()
    barrier()
    ev.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms_inflight = sum(a.elapsed_time(b) for a, b in ev) / max(1, len(ev))
    # Kernel duration for the roofline: with frames in flight a launch's events also span the wait
    # for the CUs the previous frame still holds, so the same launch (this rank's share of the
    # frame, same slot and LPT order) is timed alone, back to back, right after the timed region.
    ev.clear()
    sl0 = slots[0]
    n_iso = max(2, min(args.steps, 5))
    for _ in range(n_iso):
        with torch.cuda.stream(sl0.stream):
            if split == "samples":
                if sl0.dr.spp_r:
                    sl0.dr.render_full(sl0.dr.number, sl0.dr.spp_r, sl0.dr.accum, sl0.dr.out)
            else:
                sl0.dr.render_band(sl0.dr.rows, sl0.dr.accum[: sl0.dr.n], sl0.dr.out[: sl0.dr.n])
        torch.cuda.synchronize()
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / max(1, len(ev))
    # the per-frame rebuild alone (host build + upload), outside the timed region
    torch.cuda.synchronize()
    tb = time.perf_counter()
    renderer.set_scene(scene)
    torch.cuda.synchronize()
    build_ms = (time.perf_counter() - tb) * 1e3
    st = renderer.stats()   # last frame's counters on this rank

    samples_per_step = W * H * spp
    value = samples_per_step * args.steps / elapsed / 1e6

    # Algorithmic work of one launch on this rank, counted by the instrumented build of the same
    # kernel (identical image, same traversal; outside the timed region).
    local_rows = len(dr.rows_np) if split == "strips" else (H if dr.spp_r else 0)
    local_spp = spp if split == "strips" else dr.spp_r
    cnt_opts = rtvk.make_options(accel=accel, count_tests=True)
    cnt_opts.reserved[1] = args.walk
    cnt_spp = max(1, min(local_spp, args.count_spp))
    if local_rows:
        acc = torch.zeros((local_rows, W, 4), dtype=torch.float32, device=dev)
        out = torch.zeros((local_rows, W, 4), dtype=torch.uint8, device=dev)
        crci = rtvk.canonical_render_call_info(cnt_spp, W, H)
        if split == "samples":
            crci.number = dr.number
        renderer.render_device(crci, acc, out, rows=dr.rows if split == "strips" else None,
                               options=cnt_opts)
        torch.cuda.synchronize()
        cs = renderer.stats()
        del acc, out
    else:
        cs = rtvk.Stats()
    scale = local_spp / cnt_spp
    flops = (cs.box_tests * FLOP_PER_BOX_TEST + cs.sphere_tests * FLOP_PER_SPHERE_TEST) * scale
    achieved = flops / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0

    result = None
    if rank == 0:
        traffic = None
        tf = ROOT / "profiles" / "pmc_traffic.json"
        if tf.exists():
            try:
                tj = json.loads(tf.read_text())
                key = f"{args.accel}-{W}x{H}-{spp}spp-grid{args.grid}-n{world}"
                traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
            except (ValueError, OSError):
                traffic = None
        roof = {"bound": "valu-fp32", "achieved": round(achieved, 3), "peak": VALU_FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / VALU_FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                "kernel": ("rt_trace_brute_kernel" if accel != 2 else
                           "rt_trace_top_kernel (LDS treelet + L2 subtrees)" if renderer.scene_array(8)["device_built"]
                           else "rt_trace_lbvh_kernel (octant LDS walk)"),
                "kernel_ms": round(kernel_ms, 4),
                "kernel_timing": f"{n_iso} launches of this frame timed alone after the timed region "
                                 "(HIP events on the launch stream); with frames in flight a launch "
                                 f"spans {kernel_ms_inflight:.2f} ms including the wait for the previous "
                                 "frame's CUs",
                "flop_per_launch": int(flops), "box_tests": int(cs.box_tests * scale),
                "sphere_tests": int(cs.sphere_tests * scale),
                "flop_model": "20/box test + 23/sphere test (SURVEY.md 8(d)); counts from the "
                              f"instrumented build of the same kernel at {cnt_spp} spp"
                              + (f", x{scale:g}" if scale != 1 else "")}
        if accel == 2:   # the other fraction SURVEY.md 8(d) asks for: the LBVH's own bytes, from LDS
            lds_bytes = (cs.box_tests * BYTES_PER_BOX_TEST + cs.sphere_tests * BYTES_PER_SPHERE_TEST) * scale
            lds_tbps = lds_bytes / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
            roof["lds"] = {"achieved": round(lds_tbps, 3), "peak": round(LDS_PEAK_TBPS, 1), "unit": "TB/s",
                           "frac": round(lds_tbps / LDS_PEAK_TBPS, 4), "bytes_per_launch": int(lds_bytes),
                           "model": "32 B per box test + 16 B per sphere test (node and leaf records; "
                                    "from L2 instead of LDS below the treelet of trees too big for LDS)"}
        valu = _pmc_record(ROOT / "profiles" / "pmc_valu.json", f"{args.accel}-{W}x{H}-{spp}spp-grid{args.grid}-n{world}")
        if valu:
            roof["valu_issue_busy"] = valu.get("valu_issue_busy")
            roof["lane_util"] = valu.get("lane_util")
        result = {
            "metric": "Msamples/s (1920x1080 RTIOW scene, depth 50)",
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: canonical scene generateRandomScene(t=0), {len(scene)} spheres, "
                    "camera (13,11,-3) -> origin, global per-pixel seeds TEA(TEA(x,y),0)",
            "config": {"workload": f"rtiow-{W}x{H}-{spp}spp-depth50"
                                   + (f" (BASELINE config {args.config})" if args.config else
                                      " (BASELINE config 2 input)" if (W, H, spp, args.grid) == (1920, 1080, 100, 11) else ""),
                       "width": W, "height": H, "spp": spp, "depth": 50, "spheres": len(scene),
                       "accel": args.accel,
                       "parallelism": (f"sample-split x{world} (number+rank) + rccl all-to-all row reduction "
                                       "+ gather" if split == "samples" else f"row-strips x{world} + rccl gather"),
                       "frames_in_flight": len(slots)},
            "segments_per_sample": round(st.segments / max(1, st.samples), 4),
            "scene_setup_ms": round(t_scene * 1e3, 2),
            "scene_build_ms": round(build_ms, 3),
            "tree": "device-lbvh" if renderer.scene_array(8)["device_built"] else "host-sah",
            "msegments_per_s": round(st.segments / max(1, st.samples) * value, 2),
            "roofline": roof,
            "context": {"reference_rx6800xt_vulkan_rt_msamples": 1658.9,
                        "source": "README.md:57,61 via BASELINE.md (different GPU, HW RT cores)"},
        }
    # Side measurement: brute force (BASELINE config 2 as specified: no BVH), N = 1 only.
    if world == 1 and not args.no_brute_line and not args.profile and accel != abi.RT_ACCEL_BRUTE:
        bopts = rtvk.make_options(accel=abi.RT_ACCEL_BRUTE)
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
        renderer.render_device(rci, acc, out, options=bopts)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 2
        stream = torch.cuda.current_stream()
        e0.record(stream)
        for _ in range(reps):
            renderer.render_device(rci, acc, out, options=bopts)
        e1.record(stream)
        torch.cuda.synchronize()
        bms = e0.elapsed_time(e1) / reps
        bst = renderer.stats()
        bflops = bst.segments * len(scene) * FLOP_PER_SPHERE_TEST
        result["brute_force"] = {
            "value": round(samples_per_step / (bms * 1e-3) / 1e6, 2), "unit": "Msamples/s",
            "kernel_ms": round(bms, 3),
            "roofline": {"bound": "valu-fp32", "achieved": round(bflops / (bms * 1e-3) / 1e12, 3),
                         "peak": VALU_FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(bflops / (bms * 1e-3) / 1e12 / VALU_FP32_PEAK_TFLOPS, 4)}}
        del acc, out
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile:
        fa, fo = (slots[0].dr.accum[: slots[0].dr.n], slots[0].dr.out[: slots[0].dr.n]) if split == "strips" \
            else (None, None)   # at one rank the strips frame is the whole frame in row order
        result["cpu_baseline"] = cpu_baseline(W, H, spp, fa.cpu().numpy() if fa is not None else None,
                                              fo.cpu().numpy() if fo is not None else None)
    if rank == 0:
        print(json.dumps(result), flush=True)
    for sl in slots:
        sl.renderer.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
