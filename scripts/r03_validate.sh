#!/bin/bash
# Round-3 validation on the GPU box: the full -m gpu suite, smoke, then the bench lines of BASELINE
# configs 3 (default) and 5. Outputs gpurun_out/r03v_*. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03v}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench_config3.json 2> gpurun_out/${TAG}_bench_config3.err
rc=$?; tail -c 400 gpurun_out/${TAG}_bench_config3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err
rc=$?; tail -c 400 gpurun_out/${TAG}_bench_config5.json; exit $rc
