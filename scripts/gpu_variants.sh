#!/bin/bash
# Variant A/B session on the GPU box: quick parity gate on the default build, then timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "golden or vs_oracle" > gpurun_out/variants_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/variants_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/perf_variants.py "$@" ray-tracing-gpu-vulkan_amd/lib/variants/*.so > gpurun_out/variants.log 2>&1
rc=$?; cat gpurun_out/variants.log | tail -30; exit $rc
