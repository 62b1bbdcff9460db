#!/bin/bash
# Round-3 final validation on the GPU box at the shipped build: the full -m gpu suite, smoke, the
# rocprofv3 round profiles (kernel-trace stats + PMC passes) of BASELINE configs 3 and 5, then the
# bench lines of both with the fresh, hash-stamped PMC record. Outputs gpurun_out/${TAG}_*,
# gpurun_out/round${TAG}_c{3,5}/. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03z}
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
fi
rm -f gpurun_out/profiles_new/pmc.json
CONFIG=3 TAG=$TAG bash scripts/round_profile.sh || exit $?
CONFIG=5 TAG=$TAG bash scripts/round_profile.sh || exit $?
cp gpurun_out/profiles_new/pmc.json profiles/pmc.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench_config3.json 2> gpurun_out/${TAG}_bench_config3.err
rc=$?; tail -c 400 gpurun_out/${TAG}_bench_config3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err
rc=$?; tail -c 400 gpurun_out/${TAG}_bench_config5.json; exit $rc
