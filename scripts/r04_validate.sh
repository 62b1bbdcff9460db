#!/bin/bash
# Round-4 validation on the GPU box: the -m gpu suite, smoke (with its on-box rebuild check), the
# default bench line (config 3 + config 5 side line + both-stream cpu_baseline), then config 5
# through rt_multi on one GPU (the step overhead of the stream-ordered scene path). Outputs
# gpurun_out/${TAG}_*. An ordinary test failure does not stop the run; a time limit, abort or
# crash (exit status >= 124) does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04a}
STEPS=${STEPS:-5}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; fatal $rc smoke
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 600 gpurun_out/${TAG}_bench.json; fatal $rc bench
timeout -k 10 300 python bench.py --config 5 --path multi --gpus 1 --steps 3 --warmup 2 --no-cpu-baseline --no-rebuild-check > gpurun_out/${TAG}_bench_c5_multi.json 2> gpurun_out/${TAG}_bench_c5_multi.err
rc=$?; tail -c 300 gpurun_out/${TAG}_bench_c5_multi.json; fatal $rc bench_c5_multi
timeout -k 10 120 python scripts/grid_cells.py > gpurun_out/${TAG}_grid_cells.json 2>&1
rc=$?; cat gpurun_out/${TAG}_grid_cells.json; fatal $rc grid_cells
echo done
