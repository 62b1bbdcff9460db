#!/bin/bash
# One GPU session: the GPU test suite (or a subset, PYTEST_K), then an interleaved A/B of the
# default build against lib/variants/*.so (scripts/perf_variants.py, bit-exact gate built in).
# Stops at the first failing step. Usage: scripts/gpu_ab.sh "<perf_variants args>" ["<perf args 2>"]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PYTEST_K-all}" ]; then
    K=(); [ "${PYTEST_K:-all}" != "all" ] && K=(-k "$PYTEST_K")
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "${K[@]}" \
        > gpurun_out/ab_pytest.log 2>&1
    rc=$?; tail -3 gpurun_out/ab_pytest.log
    [ $rc -eq 0 ] || exit $rc
fi
i=0
for a in "$@"; do
    i=$((i+1))
    timeout -k 10 400 python -u scripts/perf_variants.py $a ray-tracing-gpu-vulkan_amd/lib/variants/*.so \
        > gpurun_out/ab_$i.log 2>&1
    rc=$?; echo "== ab $i ($a) rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$i.log | tail -12
    [ $rc -eq 0 ] || exit $rc
done
