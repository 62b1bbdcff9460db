"""The path's host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (the
reference has no sanitizer or validation run, src/vulkan.h:51): tests/native/sanitize_harness.cpp
drives the CPU oracle, the host LBVH / grid builders (csrc/rt_bvh.cpp, rt_grid.cpp) and the
multi-device partition, balancer and frame plan (csrc/rt_plan.cpp) over configs 3 and 5's scenes
and the edge scenes of tests/test_gpu_build.py; any sanitizer report or failed check fails the
test. CPU only (g++)."""
import shutil
import subprocess
from pathlib import Path

import pytest

NATIVE = Path(__file__).resolve().parent / "native"


@pytest.mark.timeout(900)
def test_host_code_clean_under_asan_ubsan():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    r = subprocess.run(["make", "-s", "-C", str(NATIVE), "sanitize"], capture_output=True, text=True, timeout=880)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-4000:]
    assert "checks passed (ASan + UBSan)" in r.stdout
    assert "runtime error" not in log and "AddressSanitizer" not in log, log[-4000:]
