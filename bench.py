#!/usr/bin/env python3
"""bench.py — Msamples/s of the MI355X path tracer on the canonical RTIOW scene (BASELINE.json).

One step = one frame of the hot path: every pixel of the image traced at `spp` samples, depth 50,
on the canonical scene (generateRandomScene(t=0): 488 spheres, camera (13,11,-3) -> origin),
rebuilding the acceleration structure as the reference does every frame. Default workload:
BASELINE config 3 (1920x1080, 10 000 spp, LBVH + persistent threads); on N GPUs the same frame is
tiled into row-exact strips over the ranks, re-dealt from their kernel times, and gathered to
rank 0 over RCCL (config 4 at N = 8):
strong scaling. `--config 2` (100 spp, brute force) and `--config 5` (3840x2160, 99 860 spheres,
1 000 spp) select the other BASELINE configs.

Random stream (`--rng`): "hash" (default; RT_RNG_SAMPLE_HASH, the north star's counter-based RNG:
per-sample LCG starts, fixed-point sums, samples of a pixel split into chunks over the lanes) or
"stream" (the reference's per-pixel LCG stream). Both are bit-exact against the CPU oracle; the
N = 1 line also times the other stream on the same frame (`reference_stream`).

Launch modes (the line's config.path names the one that ran):
  python bench.py [--gpus 1 --steps 3 --warmup 1]         single: one Renderer on one GPU
  python bench.py --gpus N                                 multi: rt_multi over N GPUs in ONE process
        (the C-ABI path behind the reference's ray_trace(gpu_count): ncclCommInitAll, strips, RCCL
        gather to GPU 0); exits non-zero when fewer than N GPUs are visible
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
                                                           per-process: one rank per GPU, RCCL gather
        to rank 0 (rtvk.dist); exits non-zero when WORLD_SIZE != --gpus
At N > 1 the line carries n1_check: the gathered frame against the same frame rendered on one GPU.
Rank 0 prints one JSON line (DESIGN.md §6 explains every field).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))

VALU_FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, vector FP32 (256 CU x 4 SIMD x 64 FLOP/clk x 2.4 GHz)
FLOP_PER_SPHERE_TEST = 23
FLOP_PER_BOX_TEST = 20
BYTES_PER_BOX_TEST = 32         # bytes/sample = S·(B·32 + T·16), read from LDS
BYTES_PER_SPHERE_TEST = 16
# Uniform-grid walk: a cell step recomputes one boundary's t, ((g + c·cs) - o)·(1/d)
# (fma, sub, mul) and reads the cell's two offsets; the instrumented build counts cell steps where
# the tree walk counts box tests.
FLOP_PER_CELL_STEP = 3
BYTES_PER_CELL_STEP = 8
LDS_PEAK_TBPS = 256 * 256 * 2.4e9 / 1e12   # ds_read_b128: 256 B/clk/CU x 256 CU x 2.4 GHz

CONFIGS = {   # BASELINE.json configs: width, height, spp, grid half extent, accel
    2: (1920, 1080, 100, 11, "brute"),
    3: (1920, 1080, 10000, 11, "lbvh"),
    4: (1920, 1080, 10000, 11, "lbvh"),
    5: (3840, 2160, 1000, 158, "lbvh"),
}


def host_cpus() -> dict:
    """CPUs this process may use (affinity, capped by a cgroup CPU quota) and the machine's."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"threads": max(1, min(aff, quota) if quota else aff), "affinity": aff, "cgroup_quota": quota,
            "nproc": os.cpu_count(), "model": model}


def _psnr(a, b) -> float | str:
    import numpy as np
    mse = float(np.mean((a[..., :3].astype(np.float64) - b[..., :3]) ** 2))
    return "inf" if mse == 0.0 else round(float(10.0 * np.log10(255.0 ** 2 / mse)), 2)


def cpu_baseline(width: int, height: int, spp: int, grid: int, rng_mode: int, gpu_accum=None, gpu_rgba8=None,
                 other=None, target_s: float = 12.0) -> dict:
    """The CPU oracle (C++ restatement of the shaders, brute-force closest hit) on this host's
    cores. Config 1 (1920x1080, 1 spp) is timed as a full frame, median of 3, and once more at 16
    spp (the rate is spp-independent). The reported value is a bounded sample of the
    bench frame itself: 8 blocks of pixels at its full spp, spread over the image, sized to
    ~`target_s` of CPU work. Parity: the same pixels of the GPU's bench frame (numpy [H, W, 4]) are
    compared with the oracle's, bit for bit (BASELINE.json's "PSNR vs CPU ref"). `other` = (accum,
    rgba8, rng_mode) of the same frame in the other random stream (the bench's side line): its
    pixels are checked the same way, and when it is the reference's per-pixel LCG stream also
    against the oracle's literal readings of the GLSL (LIT_RINT: shader.rint:46-55 as written;
    LIT_ALL: every dot / normalize too): the north star's "PSNR >= 50 dB vs
    reference at identical seed", measured on the headline frame."""
    import numpy as np
    from oracle import oracle
    oracle.build()
    sc = oracle.generate_scene(0.0, grid)
    cpus = host_cpus()
    threads = cpus["threads"]
    canon = oracle.generate_scene(0.0)
    c1 = []
    for _ in range(3):
        t0 = time.perf_counter()
        oracle.render(canon, oracle.render_call_info(1, 1920, 1080), 1920, 1080, threads=threads)
        c1.append(time.perf_counter() - t0)
    t1 = sorted(c1)[1]
    rate = 1920 * 1080 / t1   # samples/s on the canonical scene at 1 spp (spp-independent)
    t0 = time.perf_counter()
    oracle.render(canon, oracle.render_call_info(16, 1920, 1080), 1920, 1080, threads=threads)
    t16 = time.perf_counter() - t0
    rate16 = 1920 * 1080 * 16 / t16
    # blocks of nr rows x bw pixels, evenly spread (the oracle threads over runs of 8 pixels)
    nr = 16
    cost_scale = max(1.0, len(sc) / 488.0)   # brute force: cost per sample ~ sphere count
    pixels = max(nr, int(rate * target_s / cost_scale / max(1, spp)))
    n_blocks = 8
    bw = max(1, min(width, pixels // (n_blocks * nr)))
    ys = np.linspace(0, height - nr, n_blocks).round().astype(int)
    xs = np.linspace(0, width - bw, n_blocks).round().astype(int)[::-1]

    def blocks(rng, lit=oracle.LIT_CONTRACT):
        """The oracle's render of the blocks: (accum, rgba8, seconds, samples, stats)."""
        accs, outs, dt, st = [], [], 0.0, [0, 0, 0]
        for y, x in zip(ys, xs):
            rows = np.arange(y, y + nr, dtype=np.uint32)
            t0 = time.perf_counter()
            acc, out, s = oracle.render(sc, oracle.render_call_info(spp, width, height, (int(x), 0)), bw, nr,
                                        rows=rows, opts=oracle.options(rng_mode=rng, lit=lit), threads=threads)
            dt += time.perf_counter() - t0
            accs.append(acc)
            outs.append(out)
            st = [a + b for a, b in zip(st, s)]
        return np.concatenate(accs), np.concatenate(outs), dt, n_blocks * nr * bw * spp, st

    def gpu_blocks(a):
        return np.concatenate([a[y:y + nr, x:x + bw] for y, x in zip(ys, xs)])

    acc, out, dt, samples, st = blocks(rng_mode)
    stream_name = {0: "reference", 2: "hash"}.get(rng_mode, str(rng_mode))
    res = {"value": round(samples / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "nproc": cpus["nproc"], "cpu_model": cpus["model"], "affinity": cpus["affinity"],
           "cgroup_quota": cpus["cgroup_quota"],
           "sample": f"{n_blocks} blocks of {nr} rows x {bw} px of the bench frame ({width}x{height}, {spp} spp, "
                     f"depth 50, {len(sc)} spheres, {stream_name} stream), brute-force closest hit, {threads} "
                     f"threads, {dt:.2f} s; config 1 frame (1920x1080, 1 spp, canonical scene) median of 3 "
                     f"{t1:.3f} s = {rate / 1e6:.3f} Msamples/s; at 16 spp {t16:.2f} s = {rate16 / 1e6:.3f} "
                     f"Msamples/s; {st[0] / max(1, st[1]):.3f} segments/sample",
           "config1_frame_s": round(t1, 3), "config1_runs": [round(v, 3) for v in c1],
           "config1_msamples_per_s": round(rate / 1e6, 4), "spp16_frame_s": round(t16, 3),
           "spp16_msamples_per_s": round(rate16 / 1e6, 4),
           "spp16_over_spp1": round(rate16 / rate, 3)}   # 1 spp carries the per-frame cost (threads, seeds) alone
    if gpu_accum is not None:
        ga, go = gpu_blocks(gpu_accum), gpu_blocks(gpu_rgba8)
        res["parity"] = {"pixels": int(n_blocks * nr * bw), "stream": stream_name,
                         "accum_bit_exact": bool(np.array_equal(ga, acc)),
                         "rgba8_equal": bool(np.array_equal(go, out)), "psnr_db": _psnr(go, out)}
        if other is not None:
            o_acc, o_px, o_rng = other
            oa, oo, odt, _, _ = blocks(o_rng)
            ga, go = gpu_blocks(o_acc), gpu_blocks(o_px)
            leg = {"stream": {0: "reference", 2: "hash"}.get(o_rng, str(o_rng)),
                   "accum_bit_exact": bool(np.array_equal(ga, oa)), "rgba8_equal": bool(np.array_equal(go, oo)),
                   "psnr_db": _psnr(go, oo), "cpu_s": round(odt, 2)}
            if o_rng == 0:
                leg["vs_literal_glsl"] = {}
                for name, lit in (("rint", oracle.LIT_RINT), ("all", oracle.LIT_ALL)):
                    la, lo, ldt, _, _ = blocks(0, lit)
                    leg["vs_literal_glsl"][name] = {
                        "psnr_db": _psnr(go, lo), "rgba8_identical": round(float(np.mean(np.all(go[..., :3] == lo[..., :3], -1))), 4),
                        "accum_bit_identical": round(float(np.mean(np.all(ga[..., :3] == la[..., :3], -1))), 4),
                        "cpu_s": round(ldt, 2)}
                leg["vs_literal_glsl"]["what"] = (
                    "the GPU's reference-stream frame (identical seed) against the oracle reading shader.rint:46-55 "
                    "as written (rint) and every dot / normalize as written too (all); north star: >= 50 dB")
            res["parity"]["reference_stream" if o_rng == 0 else "hash_stream"] = leg
    return res


def lib_sha256() -> str:
    from rtvk import abi
    return hashlib.sha256(Path(abi.LIB_PATH).read_bytes()).hexdigest()[:16]


def pmc_record(key: str, sha: str) -> dict:
    """rocprofv3 --pmc summary of this workload (scripts/pmc_to_json.py), used only when it was
    measured on this exact library build (its sha256 prefix)."""
    path = ROOT / "profiles" / "pmc.json"
    try:
        rec = json.loads(path.read_text()).get(key)
    except (OSError, ValueError):
        rec = None
    if not rec:
        return {"pmc": f"no PMC record for {key} in profiles/pmc.json"}
    if rec.get("lib_sha256") != sha:
        return {"pmc": f"stale: profiles/pmc.json {key} measured on build {rec.get('lib_sha256')}, this build is {sha}"}
    return {k: rec[k] for k in ("valu_issue_busy", "lane_util", "hbm_bytes_per_launch", "kernel_ms", "l2_hit_rate")
            if k in rec}


WALK_NAMES = {   # rt_debug_launch_info form -> (kernel, walk)
    "lbvh-octant-lds": ("rt_trace_lds_kernel<8 octant copies>", "LBVH, 8 octant node copies staged in LDS"),
    "lbvh-lds": ("rt_trace_lds_kernel<1 copy>", "LBVH, one node copy staged in LDS"),
    "lbvh-treelet": ("rt_trace_top_kernel", "LBVH, LDS treelet over L2 subtrees"),
    "lbvh-global": ("rt_trace_global_kernel", "LBVH, every node from L2"),
    "grid-lds": ("rt_trace_grid_kernel<grid in LDS>", "uniform grid (3D DDA), staged in LDS"),
    "grid-lds-rec": ("rt_trace_grid_kernel<grid + shading records in LDS>",
                     "uniform grid (3D DDA) staged in LDS, with the winner's gate and shading records"),
    "grid-global": ("rt_trace_grid_kernel<grid from L2>", "uniform grid (3D DDA), from L2"),
    "grid-lds-coop": ("rt_trace_grid_kernel<grid in LDS, wave-cooperative>",
                      "uniform grid (3D DDA) staged in LDS, reference tests spread over the wave's lanes"),
    "grid-global-coop": ("rt_trace_grid_kernel<grid from L2, wave-cooperative>",
                         "uniform grid (3D DDA) from L2, reference loads and tests spread over the wave's lanes"),
}


def roofline_block(cs, scale, form: str, kernel_ms: float, step_ms: float, n_gpus: int, sha: str, pmc: dict,
                   basis: str) -> dict:
    """VALU FP32 roofline of the dominant (trace) kernel: algorithmic FLOP of one launch (counts
    of the instrumented build x scale) / the launch's duration measured inside the timed region."""
    grid_walk = form.startswith("grid")
    flop_step = FLOP_PER_CELL_STEP if grid_walk else FLOP_PER_BOX_TEST
    bytes_step = BYTES_PER_CELL_STEP if grid_walk else BYTES_PER_BOX_TEST
    flops = (cs.box_tests * flop_step + cs.sphere_tests * FLOP_PER_SPHERE_TEST) * scale
    peak = VALU_FP32_PEAK_TFLOPS * n_gpus
    achieved = flops / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
    roof = {"bound": "valu-fp32", "achieved": round(achieved, 3), "peak": round(peak, 1), "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": pmc.get("hbm_bytes_per_launch"),
            "kernel": WALK_NAMES.get(form, (form,))[0], "kernel_ms": round(kernel_ms, 4), "frac_basis": basis,
            "frac_per_step": round(flops / (step_ms * 1e-3) / 1e12 / peak, 4),
            "flop_per_launch": int(flops),
            ("cell_steps" if grid_walk else "box_tests"): int(cs.box_tests * scale),
            "sphere_tests": int(cs.sphere_tests * scale),
            "flop_model": (f"{flop_step}/{'grid cell step' if grid_walk else 'box test'} + 23/sphere test "
                           f"(SURVEY.md 8(d)); counts from the instrumented build of the same kernel"
                           + (f", x{scale:g} to the frame's spp" if scale != 1 else "")),
            "lib_sha256": sha}
    roof.update({k: v for k, v in pmc.items() if k in ("valu_issue_busy", "lane_util", "pmc", "l2_hit_rate")})
    if "valu_issue_busy" in pmc and "lane_util" in pmc:
        # every executed lane-op (traversal control, shading, sampling included) against peak
        roof["valu_lane_frac"] = round(pmc["valu_issue_busy"] * pmc["lane_util"], 4)
    if pmc.get("hbm_bytes_per_launch") and kernel_ms > 0:   # HBM GB/s against 8 TB/s
        gbs = pmc["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9
        roof["hbm"] = {"achieved": round(gbs, 1), "peak": 8000.0 * n_gpus, "unit": "GB/s",
                       "frac": round(gbs / (8000.0 * n_gpus), 5),
                       "basis": "PMC 2 x FETCH_SIZE + WRITE_SIZE per launch / the launch's duration"}
    lds_bytes = (cs.box_tests * bytes_step + cs.sphere_tests * BYTES_PER_SPHERE_TEST) * scale
    lds_tbps = lds_bytes / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
    roof["lds"] = {"achieved": round(lds_tbps, 3), "peak": round(LDS_PEAK_TBPS * n_gpus, 1), "unit": "TB/s",
                   "frac": round(lds_tbps / (LDS_PEAK_TBPS * n_gpus), 4), "bytes_per_launch": int(lds_bytes),
                   "model": (f"{bytes_step} B per {'cell step' if grid_walk else 'box test'} + 16 B per sphere test "
                             "(from L2 instead of LDS for walks whose structure does not fit LDS)")}
    return roof


def config5_line(dev, steps: int, warmup: int, sha: str, count_spp: int = 20, oracle_check: bool = True) -> dict:
    """BASELINE config 5 on this GPU: 3840x2160, 99 860 spheres (generateRandomScene grid 316x316),
    1 000 spp, the counter-based stream; every frame rebuilds the scene on the device (Morton LBVH +
    grid, rt_build.hip) as the reference rebuilds BLAS/TLAS, then renders it (grid walked from L2).
    Timed like the headline (frames back to back between syncs, after two untimed frames that
    allocate both scene arenas); the trace kernel from the
    library's HIP events; image checks: a 64-row band through the default walk equals the LDS
    treelet walk bit for bit, and 4 blocks of the timed frame equal the CPU oracle bit for bit."""
    import numpy as np
    import torch

    import rtvk
    from rtvk import abi
    W, H, spp, grid = CONFIGS[5][:4]
    scene = rtvk.generateRandomScene(0.0, grid)
    r = rtvk.Renderer(dev.index)
    stream = torch.cuda.Stream(device=dev)
    opts = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=abi.RT_RNG_SAMPLE_HASH)
    rci = rtvk.canonical_render_call_info(spp, W, H)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)

    def frame():
        with torch.cuda.stream(stream):
            r.set_scene(scene, stream=stream)
            r.render_device(rci, acc, out, options=opts, stream=stream)

    for _ in range(max(1, warmup)):
        frame()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        frame()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ks = r.kernel_times(steps)
    kernel_ms = sum(ks) / max(1, len(ks))
    step_ms = elapsed / steps * 1e3
    info = r.launch_info()
    device_built = r.scene_array(8)["device_built"]
    frame_np = (acc.cpu().numpy(), out.cpu().numpy())
    st = r.stats()
    cnt = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=abi.RT_RNG_SAMPLE_HASH, count_tests=True)
    r.render_device(rtvk.canonical_render_call_info(count_spp, W, H), acc, out, options=cnt, stream=stream)
    torch.cuda.synchronize(dev)
    cs = r.stats()
    key = f"lbvh-hash-{W}x{H}-{spp}spp-grid{grid}-n1"
    roof = roofline_block(cs, spp / count_spp, info["form"], kernel_ms, step_ms, 1, sha, pmc_record(key, sha),
                          f"mean trace-kernel duration of the {len(ks)} timed launches (HIP events on the launch stream)")
    # walk check: a 64-row band, default walk (grid from L2) vs the LDS treelet over L2 subtrees
    y0 = 1056
    band = rtvk.canonical_render_call_info(spp, W, H)
    band.offset.y = y0
    ba = [torch.zeros((64, W, 4), dtype=torch.float32, device=dev) for _ in range(2)]
    bo = [torch.zeros((64, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
    forms = []
    for i, form in enumerate((0, 8)):
        o = rtvk.make_options(accel=abi.RT_ACCEL_LBVH, rng_mode=abi.RT_RNG_SAMPLE_HASH)
        o.reserved[1] = form
        r.render_device(band, ba[i], bo[i], options=o, stream=stream)
        torch.cuda.synchronize(dev)
        forms.append(r.launch_info()["form"])
    band_equal = bool(torch.equal(ba[0], ba[1]) and torch.equal(bo[0], bo[1]))
    band_vs_frame = bool(np.array_equal(ba[0].cpu().numpy(), frame_np[0][y0:y0 + 64]))
    res = {"workload": "BASELINE config 5: 3840x2160, 99 860 spheres, 1000 spp, depth 50, hash stream, "
                       "device LBVH + grid rebuilt every frame",
           "value": round(W * H * spp * steps / elapsed / 1e6, 2), "unit": "Msamples/s", "steps": steps,
           "warmup": warmup, "ms_per_step": round(step_ms, 3), "kernel_ms": round(kernel_ms, 3),
           "step_minus_kernel_ms": round(step_ms - kernel_ms, 3),
           "accel": info["form"], "structure_build": "device" if device_built else "host",
           "sample_chunks": info["chunks"], "head_chunks": info["head_chunks"],
           "segments_per_sample": round(st.segments / max(1, st.samples), 4), "roofline": roof,
           "walk_check": {"rows": f"{y0}..{y0 + 63}", "forms": forms, "bit_equal": band_equal,
                          "band_equals_timed_frame": band_vs_frame}}
    if oracle_check:
        from oracle import oracle
        oracle.build()
        sc = oracle.generate_scene(0.0, grid)
        same_a = same_o = True
        nb, bh, bw = 4, 4, 8
        t0 = time.perf_counter()
        for y, x in zip(np.linspace(0, H - bh, nb).round().astype(int), np.linspace(0, W - bw, nb).round().astype(int)):
            rows = np.arange(y, y + bh, dtype=np.uint32)
            oa, oo, _ = oracle.render(sc, oracle.render_call_info(spp, W, H, (int(x), 0)), bw, bh, rows=rows,
                                      opts=oracle.options(rng_mode=abi.RT_RNG_SAMPLE_HASH), threads=host_cpus()["threads"])
            same_a &= bool(np.array_equal(frame_np[0][y:y + bh, x:x + bw], oa))
            same_o &= bool(np.array_equal(frame_np[1][y:y + bh, x:x + bw], oo))
        res["oracle_check"] = {"pixels": nb * bh * bw, "accum_bit_exact": same_a, "rgba8_equal": same_o,
                               "cpu_s": round(time.perf_counter() - t0, 2),
                               "what": f"{nb} blocks of {bh} rows x {bw} px of the timed frame vs the CPU oracle "
                                       "(brute force over all 99 860 spheres)"}
    r.close()
    return res


def animated_line(dev, W: int, H: int, spp: int, grid: int, rng_mode: int, frames: int = 5,
                  dt: float = 1.0 / 60.0) -> dict:
    """The reference's frame loop (src/ray_trace.cpp:579-582, :741-745): every frame regenerates the
    scene at its own t (generateRandomScene, src/scene.h:79-157: spheres 1-3 move with t,
    :94-111), rebuilds the acceleration structure and renders; t advances 1/60 s per frame. The
    tile hand-out order (LPT) of each frame comes from the previous, different frame. One untimed
    frame (t = -1/60) first, then `frames` timed frames from t = 0; the last one is checked against
    the oracle on 4 blocks of pixels."""
    import numpy as np
    import torch

    import rtvk
    r = rtvk.Renderer(dev.index)
    stream = torch.cuda.Stream(device=dev)
    opts = rtvk.make_options(accel=rtvk.abi.RT_ACCEL_LBVH, rng_mode=rng_mode)
    rci = rtvk.canonical_render_call_info(spp, W, H)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)

    def frame(t):
        sc = rtvk.generateRandomScene(t, grid)   # host generation inside the loop, as the reference
        with torch.cuda.stream(stream):
            r.set_scene(sc, stream=stream)
            r.render_device(rci, acc, out, options=opts, stream=stream)

    frame(-dt)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(frames):
        frame(k * dt)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ks = r.kernel_times(frames)
    t_last = (frames - 1) * dt
    res = {"workload": f"BASELINE config 3 frames ({W}x{H}, {spp} spp) of the reference's animated loop: "
                       f"scene regenerated at t = k/60 s, structure rebuilt, LPT order from the previous frame",
           "value": round(W * H * spp * frames / elapsed / 1e6, 2), "unit": "Msamples/s", "frames": frames,
           "ms_per_step": round(elapsed / frames * 1e3, 3), "kernel_ms": round(sum(ks) / max(1, len(ks)), 3),
           "t_s": [round(k * dt, 4) for k in range(frames)]}
    from oracle import oracle
    oracle.build()
    sc = oracle.generate_scene(t_last, grid)
    a_np, o_np = acc.cpu().numpy(), out.cpu().numpy()
    same_a = same_o = True
    nb, bh, bw = 4, 2, 8
    t1 = time.perf_counter()
    for y, x in zip(np.linspace(0, H - bh, nb).round().astype(int), np.linspace(0, W - bw, nb).round().astype(int)):
        rows = np.arange(y, y + bh, dtype=np.uint32)
        oa, oo, _ = oracle.render(sc, oracle.render_call_info(spp, W, H, (int(x), 0)), bw, bh, rows=rows,
                                  opts=oracle.options(rng_mode=rng_mode), threads=host_cpus()["threads"])
        same_a &= bool(np.array_equal(a_np[y:y + bh, x:x + bw], oa))
        same_o &= bool(np.array_equal(o_np[y:y + bh, x:x + bw], oo))
    res["oracle_check"] = {"t": t_last, "pixels": nb * bh * bw, "accum_bit_exact": same_a, "rgba8_equal": same_o,
                           "cpu_s": round(time.perf_counter() - t1, 2)}
    r.close()
    return res


def cold_call_line(W: int, H: int, spp: int, timeout_s: int = 300) -> dict:
    """One cold call of the drop-in entry point, ray_trace(spp, false, W, H, 1) (src/ray_trace.h:9-15),
    in a fresh child process with the counter-based stream (RT_RNG=hash, the headline's): HIP
    runtime start, the devices and streams (no RCCL communicator for one device), the context, the
    canonical scene's build, one frame without LPT history, the resolve and the teardown. `call_s`
    is the wall time around the call; `frame_ms` is the frame time the library itself prints
    (duration_per_frame), `create_ms` / `scene_ms` the setup it prints."""
    import re
    import subprocess
    from rtvk import abi
    code = ("import ctypes, sys, time\n"
            "lib = ctypes.CDLL(sys.argv[1])\n"
            "lib.ray_trace.argtypes = [ctypes.c_uint32, ctypes.c_bool, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]\n"
            "lib.ray_trace.restype = None\n"
            "t = time.perf_counter()\n"
            "lib.ray_trace(int(sys.argv[2]), False, int(sys.argv[3]), int(sys.argv[4]), 1)\n"
            "dt = time.perf_counter() - t\n"
            "sys.stdout.flush()\n"
            "print('CALL_S', dt, flush=True)\n")
    env = dict(os.environ, RT_RNG="hash")
    t0 = time.perf_counter()
    p = subprocess.run([sys.executable, "-c", code, str(abi.LIB_PATH), str(spp), str(W), str(H)], env=env,
                       capture_output=True, text=True, timeout=timeout_s)
    proc_s = time.perf_counter() - t0
    call = re.search(r"CALL_S ([0-9.eE+-]+)", p.stdout)
    fr = re.search(r"duration_per_frame: ([0-9.]+) ms", p.stdout)
    su = re.search(r"setup: [^0-9]*([0-9.]+) ms, scene build \+ upload ([0-9.]+) ms", p.stdout)
    if p.returncode != 0 or not call or not fr:
        return {"error": f"exit {p.returncode}", "stdout": p.stdout[-400:], "stderr": p.stderr[-400:]}
    call_s, frame_ms = float(call.group(1)), float(fr.group(1))
    parts = {"create_ms": float(su.group(1)), "scene_ms": float(su.group(2))} if su else {}
    return {"call_s": round(call_s, 4), "frame_ms": round(frame_ms, 3), "setup_s": round(call_s - frame_ms / 1e3, 4),
            **parts,
            "child_process_s": round(proc_s, 3),
            "value": round(W * H * spp / call_s / 1e6, 2), "unit": "Msamples/s",
            "what": f"ray_trace({spp}, false, {W}, {H}, 1) in a fresh process, RT_RNG=hash: HIP start, "
                    "devices and streams (create_ms), the canonical scene's build and upload (scene_ms), the first "
                    "frame without LPT history (frame_ms), teardown"}


def env_knobs() -> dict:
    """RT_* variables of this process. The library reads only RT_RNG (ray_trace(), not this bench's
    path) and RT_BVH_BUILD; rtvk reads RT_LIB (another library); bench.py reads RT_BENCH_BACKEND
    (the gloo rehearsal, marked in the line). Any other, and RT_BVH_BUILD / RT_LIB, would make the
    line describe a build or configuration other than the shipped one: refused."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("RT_")}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, choices=sorted(CONFIGS), default=3)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--grid", type=int, default=None, help="scene grid half extent (11: 488 spheres)")
    ap.add_argument("--accel", choices=["lbvh", "brute"], default=None,
                    help="lbvh: the accelerated walk the library picks (uniform grid when it fits, else "
                         "LBVH; --walk forces one); brute: every sphere per segment")
    ap.add_argument("--rng", choices=["hash", "stream"], default="hash")
    ap.add_argument("--path", choices=["auto", "single", "multi"], default="auto",
                    help="without a torch.distributed launcher: 'single' = one Renderer (one GPU), 'multi' = "
                         "rt_multi over --gpus GPUs in this process (the C-ABI path behind ray_trace(gpu_count)); "
                         "auto = single at --gpus 1, multi above")
    ap.add_argument("--count-spp", type=int, default=100,
                    help="spp of the instrumented (test-counting) launch; its counts are scaled to the frame's "
                         "spp (per-sample statistics are stationary: same scene, same streams)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-side-lines", action="store_true",
                    help="skip the other-stream, LBVH-walk and brute-force lines")
    ap.add_argument("--profile", action="store_true", help="short run for rocprofv3 (no side legs, one frame in flight)")
    ap.add_argument("--walk", type=int, default=0,
                    help="walk form (A/B only): 0 auto, 6 one LDS LBVH copy, 8 octant LBVH copies, 10 LBVH from L2, "
                         "12 grid")
    ap.add_argument("--no-config5", action="store_true", help="skip the BASELINE config 5 side line")
    ap.add_argument("--no-rebuild-check", action="store_true",
                    help="skip recompiling the library on this machine and comparing it with the shipped binary")
    ap.add_argument("--inflight", type=int, default=1,
                    help="frames in flight (single path): contexts + streams used round robin. Default 1: with "
                         "sample chunks the tail is short and a second frame only interferes (DESIGN.md §6)")
    args = ap.parse_args()
    W0, H0, spp0, grid0, accel0 = CONFIGS[args.config]
    W, H = args.width or W0, args.height or H0
    spp = args.spp if args.spp is not None else spp0
    grid = args.grid if args.grid is not None else grid0
    accel_name = args.accel or accel0
    if args.profile:
        args.inflight = 1
    knobs = env_knobs()
    bad = sorted(set(knobs) - {"RT_RNG", "RT_BENCH_BACKEND"})
    if bad:
        print(f"error: {', '.join(bad)} set: the line would not describe the shipped build / configuration "
              "(tuning goes through rt_debug_tune in tests and A/B scripts, never through the environment)",
              file=sys.stderr)
        return 2
    import numpy as np
    import torch
    import torch.distributed as dist

    import rtvk
    from rtvk import abi
    from rtvk.dist import DistributedRenderer, hip_assembler, hip_band_renderer, hip_band_timer, hip_resolver

    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if launched and world != args.gpus:
        print(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    if launched and world > 1:
        mode = "per-process"
    elif args.path == "multi" or (args.path == "auto" and args.gpus > 1):
        mode = "multi"
    else:
        mode = "single"
    n_vis = torch.cuda.device_count()
    if mode != "per-process" and args.gpus > max(1, n_vis):
        print(f"error: --gpus {args.gpus} but only {n_vis} GPU(s) visible; refusing to report a smaller run",
              file=sys.stderr)
        return 2
    if mode == "single" and args.gpus != 1:
        print("error: --path single renders on one GPU; use --gpus 1", file=sys.stderr)
        return 2
    rebuild = None
    if not args.no_rebuild_check and not args.profile and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # Build provenance: compile the library from this tree's sources on this machine and compare
        # it with the shipped binary; when they differ, the fresh binary replaces it before it loads.
        import shutil
        import __graft_entry__ as ge
        rebuild = ge.rebuild_check()
        if not rebuild["identical"]:
            shutil.copy2(rebuild["box_built"], ROOT / "ray-tracing-gpu-vulkan_amd" / "lib" / "librt_mi355x.so")
            rebuild["replaced_shipped"] = True
        shutil.rmtree(Path(rebuild.pop("box_built")).parents[2], ignore_errors=True)
    n_gpus = args.gpus
    # RCCL (backend "nccl"); RT_BENCH_BACKEND=gloo rehearses N ranks sharing the visible GPUs
    # (bands staged through host memory): a test of the N > 1 code path, never a reported number.
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, n_vis)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if mode == "per-process":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    accel = abi.RT_ACCEL_BRUTE if accel_name == "brute" else abi.RT_ACCEL_LBVH
    rng_mode = abi.RT_RNG_SAMPLE_HASH if args.rng == "hash" else abi.RT_RNG_PIXEL_STREAM
    scene = rtvk.generateRandomScene(0.0, grid)
    rci = rtvk.canonical_render_call_info(spp, W, H)
    opts = rtvk.make_options(accel=accel, rng_mode=rng_mode)
    opts.reserved[1] = args.walk
    cnt_opts = rtvk.make_options(accel=accel, rng_mode=rng_mode, count_tests=True)
    cnt_opts.reserved[1] = args.walk
    cnt_spp = max(1, min(spp, args.count_spp))
    cnt_rci = rtvk.canonical_render_call_info(cnt_spp, W, H)
    scale = spp / cnt_spp

    def sync_all():
        for d in range(n_gpus if mode == "multi" else 1):
            torch.cuda.synchronize(d if mode == "multi" else dev)

    def barrier():
        sync_all()
        if mode == "per-process":
            dist.barrier()
        sync_all()

    multi_info = None
    if mode == "multi":
        # One process drives every GPU through the C-ABI (rt_multi: ncclCommInitAll, row-exact
        # strips re-dealt from the devices' kernel times, grouped ncclSend / ncclRecv of every
        # device's rows to GPU 0, reorder there):
        # the code the reference's ray_trace(gpu_count) binds (src/ray_trace.cpp:42-105, :922-972).
        mr = rtvk.MultiRenderer(n_gpus)
        if mr.device_count != n_gpus:
            print(f"error: rt_multi opened {mr.device_count} devices, asked for {n_gpus}", file=sys.stderr)
            return 2
        acc0 = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0")
        out0 = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda:0")
        t_scene = time.perf_counter()
        mr.set_scene(scene)
        sync_all()
        t_scene = time.perf_counter() - t_scene

        def frame():
            # per-frame rebuild as the reference does (src/vulkan.h:1020-1059), then render + gather
            mr.set_scene(scene)
            mr.render(rci, acc0, out0, options=opts)
            return acc0, out0
    else:
        ev_slots = []

        class Slot:
            """One frame in flight: its own context (scene blob, counters, LPT history), stream and
            frame buffers; frames go to the slots round robin."""
            def __init__(self):
                self.renderer = rtvk.Renderer(local)
                self.stream = torch.cuda.Stream(device=dev)
                with torch.cuda.stream(self.stream):
                    # rows re-dealt between frames from every rank's kernel time and per-row work of
                    # the frame two before (rtvk.dist, rt_partition_rebalance)
                    self.dr = DistributedRenderer(W, H, dev, hip_band_renderer(self.renderer, rci, opts),
                                                  hip_assembler(self.renderer),
                                                  resolve=hip_resolver(self.renderer, spp),
                                                  timer=hip_band_timer(self.renderer))
                self.launches = 0

            def frame(self):
                # The reference rebuilds its acceleration structure every frame (src/vulkan.h:1020-1059)
                # and SURVEY.md 8(d) counts the build in the wall clock: rebuild, then render (+ gather).
                with torch.cuda.stream(self.stream):
                    self.renderer.set_scene(scene, stream=self.stream)
                    self.launches += 1
                    return self.dr.step()

        slots = [Slot() for _ in range(max(1, args.inflight if mode == "single" else 1))]
        renderer, dr = slots[0].renderer, slots[0].dr
        sync_all()
        t_scene = time.perf_counter()
        renderer.set_scene(scene)
        sync_all()
        t_scene = time.perf_counter() - t_scene
        n_frames = 0

        def frame():
            nonlocal n_frames
            r = slots[n_frames % len(slots)].frame()
            n_frames += 1
            return r

    for _ in range(max(args.warmup, 1 if mode == "multi" else len(slots))):   # LPT order, occupancy
        frame()
    barrier()
    if mode != "multi":
        for sl in slots:
            sl.launches = 0
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = frame()
    barrier()
    elapsed = time.perf_counter() - t0
    # trace-kernel durations inside the timed region (HIP events the library records around the
    # kernel on its launch stream; rt_debug_kernel_times)
    per_device_ms = None   # N > 1: mean trace-kernel ms of the timed frames per device / rank
    if mode == "multi":
        frames = mr.kernel_times(min(64, args.steps))   # per timed frame, each device
        per_frame = [max(f) for f in frames if f]
        kernel_ms = sum(per_frame) / max(1, len(per_frame))
        per_device_ms = [sum(f[d] for f in frames) / len(frames) for d in range(len(frames[0]))] if frames else []
        last_k = frames[-1] if frames else []
        k_basis = (f"mean over the {len(per_frame)} timed frames of the slowest device's trace kernel (HIP events "
                   f"on each launch stream); last frame per device: {', '.join(f'{v:.2f}' for v in last_k)} ms")
    else:
        ks = []
        for sl in slots:
            if sl.launches and sl.dr.n:
                ks += sl.renderer.kernel_times(min(64, sl.launches))
        kernel_ms = sum(ks) / max(1, len(ks))
        k_basis = (f"mean trace-kernel duration of the {len(ks)} launches of the timed region (HIP events "
                   f"recorded by the library around the kernel on its launch stream)")
        if len(slots) > 1:
            # with frames in flight a launch's events also span the wait for CUs the other slot's
            # frame holds: time 3 frames alone (one at a time) for the kernel's own duration
            for _ in range(3):
                slots[0].frame()
                sync_all()
            ks = slots[0].renderer.kernel_times(3)
            kernel_ms = sum(ks) / max(1, len(ks))
            k_basis = (f"mean trace-kernel duration of 3 frames rendered one at a time after the timed region "
                       f"(HIP events on the launch stream); the timed region had {len(slots)} frames in flight")
    if mode == "per-process":
        # every rank's kernel time (the reference records per-GPU durations and the row split of
        # every benchmark window, src/ray_trace.cpp:750-760), then the max over ranks
        cdev = dev if backend == "nccl" else torch.device("cpu")
        mine = torch.tensor([kernel_ms], dtype=torch.float64, device=cdev)
        allk = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allk, mine)
        per_device_ms = [float(v.item()) for v in allk]
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0].item()), float(t[1].item())
        k_basis += f"; max over {world} ranks"
    step_ms = elapsed / args.steps * 1e3

    # Algorithmic work of one frame, counted by the instrumented build of the same kernel
    # (identical image, same traversal; outside the timed region).
    if mode == "multi":
        st = mr.stats()
        info = None
        ca = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0")
        co = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda:0")
        mr.render(cnt_rci, ca, co, options=cnt_opts)
        sync_all()
        cs = mr.stats()
        del ca, co
        multi_info = mr.info()
        # the walk form of device 0's context (every device renders the same scene the same way)
        probe = rtvk.Renderer(0)
        probe.set_scene(scene)
        pa = torch.zeros((8, W, 4), dtype=torch.float32, device="cuda:0")
        po = torch.zeros((8, W, 4), dtype=torch.uint8, device="cuda:0")
        probe.render_device(rtvk.canonical_render_call_info(1, W, H), pa, po, options=opts)
        sync_all()
        info = probe.launch_info()
        info["chunks"] = None   # per device, chosen for its own band
        device_built = probe.scene_array(8)["device_built"]
    else:
        st = renderer.stats()   # this rank's last band
        info = renderer.launch_info()
        device_built = renderer.scene_array(8)["device_built"]
        if dr.n:
            acc = torch.zeros((dr.n, W, 4), dtype=torch.float32, device=dev)
            out = torch.zeros((dr.n, W, 4), dtype=torch.uint8, device=dev)
            renderer.render_device(cnt_rci, acc, out, rows=dr.rows, options=cnt_opts)
            sync_all()
            cs = renderer.stats()
            del acc, out
        else:
            cs = rtvk.Stats()
        if mode == "per-process":   # whole-frame counts: sum over the ranks
            t = torch.tensor([cs.box_tests, cs.sphere_tests, st.segments, st.samples], dtype=torch.float64,
                             device=dev)
            dist.all_reduce(t)
            cs = rtvk.Stats(segments=0, samples=0, box_tests=int(t[0].item()), sphere_tests=int(t[1].item()))
            st = rtvk.Stats(segments=int(t[2].item()), samples=int(t[3].item()), box_tests=0, sphere_tests=0)
    form = "brute" if accel == abi.RT_ACCEL_BRUTE else info["form"]
    # host cost of one per-frame scene call with the GPU idle (host build + upload issue for host
    # scenes; for device builds it includes the build, which in the timed loop overlaps the
    # previous frame): the per-frame setup a rank pays outside the kernel
    sync_all()
    t_sc = time.perf_counter()
    for _ in range(5):
        if mode == "multi":
            mr.set_scene(scene)
        else:
            renderer.set_scene(scene)
    scene_call_ms = (time.perf_counter() - t_sc) / 5 * 1e3
    sync_all()

    samples_per_step = W * H * spp
    value = samples_per_step * args.steps / elapsed / 1e6
    result = None
    frame_np = None
    if rank == 0:
        sha = lib_sha256()
        key = f"{accel_name}-{args.rng}-{W}x{H}-{spp}spp-grid{grid}-n{n_gpus}"
        pmc = pmc_record(key, sha)
        if accel == abi.RT_ACCEL_BRUTE:
            flops = st.segments * len(scene) * FLOP_PER_SPHERE_TEST
            peak = VALU_FP32_PEAK_TFLOPS * n_gpus
            ach = flops / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
            roof = {"bound": "valu-fp32", "achieved": round(ach, 3), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4), "traffic": pmc.get("hbm_bytes_per_launch"),
                    "kernel": "rt_trace_brute_kernel", "kernel_ms": round(kernel_ms, 4), "frac_basis": k_basis,
                    "frac_per_step": round(flops / (step_ms * 1e-3) / 1e12 / peak, 4), "lib_sha256": sha}
        else:
            roof = roofline_block(cs, scale, form, kernel_ms, step_ms, n_gpus, sha, pmc, k_basis)
        cfg_name = (f"BASELINE config {args.config}" if n_gpus == 1 or args.config not in (3, 4)
                    else f"BASELINE config {4 if n_gpus == 8 else 3} frame on {n_gpus} GPUs")
        default_shape = (W, H, spp, grid, accel_name) == CONFIGS[args.config]
        walk = "brute-force sphere list (scalar cache)" if form == "brute" else WALK_NAMES.get(form, (form, form))[1]
        if mode == "multi":
            par = (f"rt_multi (C-ABI, one process): {multi_info['devices']} GPUs, row-exact interleaved "
                   f"{multi_info['strip_rows']}-row strips re-dealt between frames from the devices' kernel times, "
                   + (f"RCCL grouped ncclSend/ncclRecv gather of every other GPU's accumulator strips to GPU 0 "
                      f"(ncclCommInitAll communicator of {multi_info['rccl_ranks']} ranks) + device reorder + "
                      f"resolve on GPU 0" if multi_info["devices"] > 1 else
                      "one GPU renders straight into the caller's buffers (no communicator, no collective)"))
        elif mode == "per-process":
            par = (f"torch.distributed ({backend}): {world} processes, one per GPU, row-exact interleaved 8-row "
                   f"strips re-dealt between frames from the ranks' kernel times (gloo exchange of per-row costs) + "
                   f"gather of the float4 accumulator rows to rank 0 + device reorder + rgba8 resolve on rank 0")
        else:
            par = "1 GPU"
        result = {
            "metric": "Msamples/s (1920x1080 RTIOW scene, depth 50)" if (W, H) == (1920, 1080)
                      else f"Msamples/s ({W}x{H} RTIOW scene, depth 50)",
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: canonical scene generateRandomScene(t=0), grid {2 * grid}x{2 * grid} "
                    f"({len(scene)} spheres), camera (13,11,-3) -> origin, global per-pixel seeds "
                    f"TEA(TEA(x,y),0), {'counter-based per-sample streams (RT_RNG_SAMPLE_HASH)' if args.rng == 'hash' else 'the reference per-pixel LCG stream'}",
            "config": {"workload": f"rtiow-{W}x{H}-{spp}spp-depth50"
                                   + (f" ({cfg_name} workload)" if default_shape else " (custom)"),
                       "width": W, "height": H, "spp": spp, "depth": 50, "spheres": len(scene),
                       "accel": form, "walk": walk,
                       "structure_build": ("device (Morton + radix sort + Karras LBVH, device grid)" if device_built
                                           else "host (binned-SAH LBVH + uniform grid), uploaded per frame"),
                       "rng": args.rng, "sample_chunks": info["chunks"],
                       "path": mode, "parallelism": par,
                       "frames_in_flight": 1 if mode == "multi" else len(slots)},
            "segments_per_sample": round(st.segments / max(1, st.samples), 4),
            "scene_setup_ms": round(t_scene * 1e3, 2),
            "scene_call_ms": round(scene_call_ms, 3),
            "msegments_per_s": round(st.segments / max(1, st.samples) * value, 2),
            "roofline": roof,
            "build": {**abi.build_info(), "env": knobs,
                      "rebuild": rebuild if rebuild is not None else "skipped"},
            **({"rehearsal": f"{backend} backend, {world} ranks sharing {n_vis} GPU(s): "
                               "code-path test, not a measurement"} if backend != "nccl" and mode == "per-process" else {}),
            "context": {"reference_rx6800xt_vulkan_rt_msamples": 1658.9,
                        "source": "README.md:57,61 via BASELINE.md (different GPU, HW RT cores)"},
        }
        fa, fo = last
        if n_gpus > 1:
            # N > 1 verifies itself: the gathered frame against this frame rendered on ONE GPU
            r1 = rtvk.Renderer(local)
            r1.set_scene(scene)
            a1 = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
            o1 = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
            r1.render_device(rci, a1, o1, options=opts)
            torch.cuda.synchronize(dev)
            fa_d, fo_d = fa.to(dev), fo.to(dev)
            result["n1_check"] = {
                "pixels": W * H, "accum_bit_equal": bool(torch.equal(fa_d, a1)),
                "rgba8_equal": bool(torch.equal(fo_d, o1)),
                "what": "gathered N-GPU frame vs the same frame rendered by one GPU (same seeds, same stream)"}
            result["rccl_ranks"] = multi_info["rccl_ranks"] if mode == "multi" else world
            r1.close()
            if per_device_ms:
                mean = sum(per_device_ms) / len(per_device_ms)
                result["per_device_kernel_ms"] = [round(v, 3) for v in per_device_ms]
                result["imbalance"] = round(max(per_device_ms) / mean, 4) if mean > 0 else None
                if mode == "multi":
                    result["rows_per_device"] = [len(p) for p in mr.partition(H)]
                    result["balance"] = mr.balance_info()
                else:
                    result["rows_per_device"] = dr.rows_per_rank()
                    result["balance"] = {"frames": dr.launches, "rebalances": dr.rebalances,
                                         "rows_moved": dr.rows_moved, "predicted_imbalance": round(dr.predicted, 5)}
                result["imbalance_basis"] = ("max / mean over devices of each device's mean trace-kernel ms over "
                                             "the timed frames (HIP events on its launch stream); rows_per_device: "
                                             "the balancer's partition after the timed frames (row-exact strips "
                                             "re-dealt from the kernel times of the frame two before)")
        if n_gpus == 1:
            frame_np = (fa.cpu().numpy(), fo.cpu().numpy())
    # Side lines (single GPU): the same frame with the other random stream and with the LBVH walk
    # (BASELINE config 3 names LBVH traversal), and BASELINE configs 2 and 5 as specified.
    other_frame = None
    if mode == "single" and not args.no_side_lines and not args.profile:
        def time_frames(o, w, h, s, n):
            a = torch.zeros((h, w, 4), dtype=torch.float32, device=dev)
            b = torch.zeros((h, w, 4), dtype=torch.uint8, device=dev)
            r = rtvk.canonical_render_call_info(s, w, h)
            renderer.render_device(r, a, b, options=o)   # warm: LPT order, occupancy
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                renderer.render_device(r, a, b, options=o)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / n, a, b
        if accel != abi.RT_ACCEL_BRUTE:
            other = abi.RT_RNG_PIXEL_STREAM if rng_mode == abi.RT_RNG_SAMPLE_HASH else abi.RT_RNG_SAMPLE_HASH
            oms, oa, ob = time_frames(rtvk.make_options(accel=accel, rng_mode=other), W, H, spp, 1)
            o_np = ob.cpu().numpy()
            other_frame = (oa.cpu().numpy(), o_np, other)
            mse = float(np.mean((o_np[..., :3].astype(np.float64) - frame_np[1][..., :3]) ** 2))
            result["reference_stream" if other == abi.RT_RNG_PIXEL_STREAM else "hash_stream"] = {
                "value": round(samples_per_step / (oms * 1e-3) / 1e6, 2), "unit": "Msamples/s",
                "kernel_ms": round(oms, 3), "rng": "stream" if other == abi.RT_RNG_PIXEL_STREAM else "hash",
                "psnr_vs_headline_frame_db": "inf" if mse == 0 else round(10 * np.log10(255 ** 2 / mse), 2),
                "note": "same frame, other random stream (two independent Monte-Carlo estimates of one picture)"}
            if form.startswith("grid"):
                lo = rtvk.make_options(accel=accel, rng_mode=rng_mode)
                lo.reserved[1] = 8   # octant LBVH copies in LDS
                lms, la, lb = time_frames(lo, W, H, spp, 1)
                linfo = renderer.launch_info()
                lcnt = rtvk.make_options(accel=accel, rng_mode=rng_mode, count_tests=True)
                lcnt.reserved[1] = 8
                a_ = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
                b_ = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
                renderer.render_device(cnt_rci, a_, b_, options=lcnt)
                torch.cuda.synchronize()
                lcs = renderer.stats()
                lroof = roofline_block(lcs, scale, linfo["form"], lms, lms, 1, result["roofline"]["lib_sha256"], {},
                                       "one frame timed alone (HIP events)")
                result["lbvh_walk"] = {
                    "workload": f"BASELINE config {args.config} frame, LBVH walk (octant node copies in LDS)",
                    "accel": linfo["form"], "value": round(samples_per_step / (lms * 1e-3) / 1e6, 2),
                    "unit": "Msamples/s", "kernel_ms": round(lms, 3),
                    "image_bit_equal_to_headline": bool(np.array_equal(la.cpu().numpy(), frame_np[0])
                                                        and np.array_equal(lb.cpu().numpy(), frame_np[1])),
                    "roofline": {k: lroof[k] for k in ("bound", "achieved", "peak", "unit", "frac", "kernel",
                                                       "box_tests", "sphere_tests", "flop_per_launch")}}
        if grid == 11:
            bw_, bh_, bspp = CONFIGS[2][:3]
            bms, _, _ = time_frames(rtvk.make_options(accel=abi.RT_ACCEL_BRUTE, rng_mode=rng_mode), bw_, bh_, bspp, 2)
            bst = renderer.stats()
            bflops = bst.segments * len(scene) * FLOP_PER_SPHERE_TEST
            result["brute_force"] = {
                "workload": "BASELINE config 2: 1920x1080, 100 spp, brute-force sphere list",
                "value": round(bw_ * bh_ * bspp / (bms * 1e-3) / 1e6, 2), "unit": "Msamples/s",
                "kernel_ms": round(bms, 3),
                "roofline": {"bound": "valu-fp32", "achieved": round(bflops / (bms * 1e-3) / 1e12, 3),
                             "peak": VALU_FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                             "frac": round(bflops / (bms * 1e-3) / 1e12 / VALU_FP32_PEAK_TFLOPS, 4)}}
        if args.config == 3 and not args.no_config5 and (W, H, spp, grid) == CONFIGS[3][:4]:
            result["config5"] = config5_line(dev, steps=5, warmup=2, sha=result["roofline"]["lib_sha256"])
        if args.config == 3 and (W, H, spp, grid) == CONFIGS[3][:4] and accel != abi.RT_ACCEL_BRUTE:
            # the reference's animated loop and one cold drop-in call, beside the warm static frames
            result["animated"] = animated_line(dev, W, H, spp, grid, rng_mode)
            result["animated"]["vs_headline"] = round(result["animated"]["value"] / result["value"], 4)
            cold = cold_call_line(W, H, spp)
            if "value" in cold:
                cold["vs_headline"] = round(cold["value"] / result["value"], 4)
            result["ray_trace_call"] = cold
            result["ray_trace_call_s"] = cold.get("call_s")
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline and not args.profile:
        result["cpu_baseline"] = cpu_baseline(W, H, spp, grid, rng_mode, frame_np[0], frame_np[1], other=other_frame)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if mode == "multi":
        mr.close()
    else:
        for sl in slots:
            sl.renderer.close()
    if mode == "per-process":
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
