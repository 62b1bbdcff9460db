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
                        "--steps", "3", "--warmup", "1"],
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
