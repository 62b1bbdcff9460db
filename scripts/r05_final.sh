#!/bin/bash
# Round-5 measurement on the GPU box at the shipped build: the whole -m gpu suite and smoke, the
# rocprofv3 round profiles (kernel-trace stats + PMC passes) of BASELINE configs 3 and 5, the default
# bench line with the fresh hash-stamped PMC record, config 3 and config 5 through rt_multi on one
# GPU, and the N = 8 band probe of config 4. Outputs gpurun_out/${TAG}_*, gpurun_out/round${TAG}_c{3,5}/,
# gpurun_out/profiles_new/pmc.json. A time limit, abort or crash (exit status >= 124) stops the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05f}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
    rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; fatal $rc smoke
fi
rm -f gpurun_out/profiles_new/pmc.json
CONFIG=3 TAG=$TAG bash scripts/round_profile.sh; rc=$?; fatal $rc profile3; [ $rc -eq 0 ] || exit $rc
CONFIG=5 TAG=$TAG bash scripts/round_profile.sh; rc=$?; fatal $rc profile5; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/profiles_new/pmc.json profiles/pmc.json
timeout -k 10 700 python bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 400 gpurun_out/${TAG}_bench.json; fatal $rc bench
timeout -k 10 300 python bench.py --path multi --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-rebuild-check \
    > gpurun_out/${TAG}_bench_multi_n1_config3.json 2> gpurun_out/${TAG}_bench_multi_n1_config3.err
rc=$?; tail -c 300 gpurun_out/${TAG}_bench_multi_n1_config3.json; fatal $rc bench_multi_c3
timeout -k 10 200 python bench.py --config 5 --path multi --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-rebuild-check \
    > gpurun_out/${TAG}_bench_c5_multi.json 2> gpurun_out/${TAG}_bench_c5_multi.err
rc=$?; tail -c 300 gpurun_out/${TAG}_bench_c5_multi.json; fatal $rc bench_c5_multi
timeout -k 10 200 python scripts/band_probe.py 8 10000 --json gpurun_out/${TAG}_band_probe_n8.json > gpurun_out/${TAG}_band_probe_n8.log 2>&1
rc=$?; tail -c 400 gpurun_out/${TAG}_band_probe_n8.log; fatal $rc band_probe
echo done
