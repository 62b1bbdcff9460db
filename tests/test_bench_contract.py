"""bench.py's output contract (one JSON line with the driver's fields, roofline and cpu_baseline),
on a tiny workload through the real library."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.gpu
def test_bench_json_line_contract():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--width", "96", "--height", "64", "--spp", "2",
                        "--steps", "3", "--warmup", "1", "--no-rebuild-check"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["higher_is_better"] is True and d["vs_baseline"] is None
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["unit"] == "Msamples/s"
    assert "workload" in d["config"] and "model" not in d["config"]
    roof = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    assert 0 < roof["frac"] < 1 and roof["achieved"] > 0
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["nproc"] >= 1 and cb["cpu_model"]
    assert d["config"]["rng"] == "hash" and "reference_stream" in d and "brute_force" in d
    assert d["roofline"]["lib_sha256"] and "frac_basis" in d["roofline"]
    assert cb["parity"]["accum_bit_exact"] and cb["parity"]["rgba8_equal"] and cb["parity"]["psnr_db"] == "inf"
    # both streams' pixels against the oracle, and the reference stream against the literal GLSL
    ref = cb["parity"]["reference_stream"]
    assert ref["accum_bit_exact"] and ref["rgba8_equal"], ref
    assert set(ref["vs_literal_glsl"]) >= {"rint", "all"}
    assert len(cb["config1_runs"]) == 3 and cb["spp16_msamples_per_s"] > 0
    assert d["build"]["env"] == {} and d["build"]["rebuild"] == "skipped"
    # honest labels: the accel named in config is the walk that ran (the roofline's kernel)
    assert d["config"]["path"] == "single" and d["config"]["accel"] in ("grid-lds-rec", "grid-lds", "lbvh-octant-lds")
    assert ("grid" in d["roofline"]["kernel"]) == d["config"]["accel"].startswith("grid")
    # the kernel is timed inside the timed region: it cannot outlast the step
    assert 0 < roof["kernel_ms"] <= d["ms_per_step"]
    assert d["build"]["built_from_tree"], d["build"]
    if d["config"]["accel"].startswith("grid"):
        assert d["lbvh_walk"]["image_bit_equal_to_headline"] and d["lbvh_walk"]["accel"] == "lbvh-octant-lds"


@pytest.mark.gpu
def test_bench_multi_path_one_gpu():
    """--path multi: the C-ABI rt_multi path (one process; strips + RCCL gather at N > 1) on the
    box's one GPU; labelled as such: one device renders straight into the caller's buffers and
    holds no communicator."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--width", "96", "--height", "64", "--spp", "2",
                        "--steps", "2", "--warmup", "1", "--path", "multi", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["config"]["path"] == "multi" and "rt_multi" in d["config"]["parallelism"]
    assert "no communicator" in d["config"]["parallelism"]
    assert d["n_gpus"] == 1 and d["value"] > 0 and 0 < d["roofline"]["kernel_ms"] <= d["ms_per_step"]


def test_bench_refuses_more_gpus_than_visible():
    """--gpus N without a launcher drives rt_multi over N GPUs; with fewer visible it fails instead
    of silently benching fewer."""
    import torch
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(max(1, n) + 1), "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 2 and "visible" in r.stderr


def test_bench_refuses_tuning_environment():
    """A tuning or library-selecting RT_* variable in the environment would make the line describe
    something other than the shipped build: bench.py refuses before rendering."""
    import os
    for var, val in (("RT_SAMPLE_CHUNKS", "7"), ("RT_LIB", "/tmp/x.so"), ("RT_BVH_BUILD", "gpu")):
        e = dict(os.environ, **{var: val})
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "1"],
                           capture_output=True, text=True, timeout=300, cwd=ROOT, env=e)
        assert r.returncode == 2 and var in r.stderr, (var, r.stderr[-500:])


def test_bench_refuses_launcher_mismatch():
    import os
    e = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=e)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
