#!/bin/bash
# Round-4 final measurement on the GPU box at the shipped build: a GPU test subset, the rocprofv3
# round profiles (kernel-trace stats + PMC passes) of BASELINE configs 3 and 5, then the default
# bench line (config 3 + config 5 side line + both-stream cpu_baseline) with the fresh,
# hash-stamped PMC record, and config 5 through rt_multi on one GPU. Outputs gpurun_out/${TAG}_*,
# gpurun_out/round${TAG}_c{3,5}/, gpurun_out/profiles_new/pmc.json. A time limit, abort or crash
# (exit status >= 124) stops the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04f}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ "${FULL:-0}" = 1 ]; then   # the whole GPU suite (~100 s) instead of the contract subset
    timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
else
    timeout -k 10 240 python -u -m pytest tests/test_gpu_contract.py tests/test_bench_contract.py -m gpu -q -x --timeout 200 \
        --timeout-method thread > gpurun_out/${TAG}_pytest_subset.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_pytest_subset.log; fatal $rc pytest
fi
rm -f gpurun_out/profiles_new/pmc.json
CONFIG=3 TAG=$TAG bash scripts/round_profile.sh; rc=$?; fatal $rc profile3; [ $rc -eq 0 ] || exit $rc
CONFIG=5 TAG=$TAG bash scripts/round_profile.sh; rc=$?; fatal $rc profile5; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/profiles_new/pmc.json profiles/pmc.json
timeout -k 10 420 python bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 400 gpurun_out/${TAG}_bench.json; fatal $rc bench
timeout -k 10 200 python bench.py --config 5 --path multi --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-rebuild-check \
    > gpurun_out/${TAG}_bench_c5_multi.json 2> gpurun_out/${TAG}_bench_c5_multi.err
rc=$?; tail -c 300 gpurun_out/${TAG}_bench_c5_multi.json; fatal $rc bench_c5_multi
echo done
