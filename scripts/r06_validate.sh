#!/bin/bash
# Round-6 validation on the GPU box: the -m gpu suite (with the logical-device multi tests), smoke,
# the N = 8 band probes with the cross-device balancer iterated on measured band times (config 4:
# 1080p / 10 000 spp; config 5: 4K / 99 860 spheres / 1 000 spp with the per-frame device rebuild),
# and a 4-rank gloo rehearsal of the per-process bench path (the balancer with real HIP timers on
# ranks sharing one GPU: a code-path test, not a number). Outputs gpurun_out/${TAG}_*. An ordinary
# test failure does not stop the run; a time limit, abort or crash (exit status >= 124) does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06a}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; fatal $rc smoke
fi
if [ "${SKIP_PROBES:-0}" != 1 ]; then
timeout -k 10 400 python scripts/band_probe.py 8 10000 --iters 6 --reps 4 --json gpurun_out/${TAG}_band_probe_c3_n8.json > gpurun_out/${TAG}_band_probe_c3_n8.log 2>&1
rc=$?; tail -c 400 gpurun_out/${TAG}_band_probe_c3_n8.log; fatal $rc band_probe_c3
timeout -k 10 300 python scripts/band_probe.py 8 1000 --width 3840 --height 2160 --grid 158 --iters 5 --reps 3 --rebuild \
    --json gpurun_out/${TAG}_band_probe_c5_n8.json > gpurun_out/${TAG}_band_probe_c5_n8.log 2>&1
rc=$?; tail -c 400 gpurun_out/${TAG}_band_probe_c5_n8.log; fatal $rc band_probe_c5
fi
if [ "${SKIP_REHEARSAL:-0}" != 1 ]; then
RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 4 --warmup 4 --spp 500 \
    > gpurun_out/${TAG}_rehearsal_n4_gloo.json 2> gpurun_out/${TAG}_rehearsal_n4_gloo.err
rc=$?; echo "gloo n4 rc=$rc"; tail -c 1200 gpurun_out/${TAG}_rehearsal_n4_gloo.json; fatal $rc rehearsal
fi
echo done
