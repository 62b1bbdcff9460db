#!/bin/bash
# Round-5 validation on the GPU box: the -m gpu suite, smoke (with its on-box rebuild check), the
# default bench line (config 3 + config 5 side line + animated loop + cold ray_trace call +
# both-stream cpu_baseline), the N = 8 band probe of config 4 at the shipped build and one PMC
# WRITE_SIZE pass over rank 0's band. Outputs gpurun_out/${TAG}_*. An ordinary test failure does
# not stop the run; a time limit, abort or crash (exit status >= 124) does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05a}
STEPS=${STEPS:-5}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; fatal $rc smoke
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
timeout -k 10 700 python bench.py --steps $STEPS --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 600 gpurun_out/${TAG}_bench.json; fatal $rc bench
fi
timeout -k 10 200 python scripts/band_probe.py 8 10000 --json gpurun_out/${TAG}_band_probe_n8.json > gpurun_out/${TAG}_band_probe_n8.log 2>&1
rc=$?; tail -c 600 gpurun_out/${TAG}_band_probe_n8.log; fatal $rc band_probe
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$(pwd)/gpurun_out/${TAG}_band_pmc" -o run -- \
    python3 scripts/band_probe.py 8 10000 --ranks 0 --reps 1 --no-full > gpurun_out/${TAG}_band_pmc.log 2>&1 < /dev/null
rc=$?; tail -c 300 gpurun_out/${TAG}_band_pmc.log; fatal $rc band_pmc
echo done
