#!/bin/bash
# Round-5: A/B of variant libraries (config 3 at 1000 spp both streams, config 5 at 100 spp), the
# gloo 2-rank rehearsal of the per-process bench path and one cold ray_trace() call. Outputs
# gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05g}
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -lt 124 ] || exit $rc
fi
SKIP_BAND=1 TAG=$TAG bash scripts/r05_ab.sh; rc=$?; [ $rc -lt 124 ] || exit $rc
if [ "${SKIP_REHEARSAL:-0}" != 1 ]; then
RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --spp 1000 \
    > gpurun_out/${TAG}_rehearsal_n2_gloo.json 2> gpurun_out/${TAG}_rehearsal_n2_gloo.err
rc=$?; echo "gloo n2 rc=$rc"; tail -c 900 gpurun_out/${TAG}_rehearsal_n2_gloo.json; [ $rc -lt 124 ] || exit $rc
fi
timeout -k 10 200 python -c "
import json, sys; sys.argv=['bench.py']; import bench
print(json.dumps(bench.cold_call_line(1920, 1080, 10000)))" > gpurun_out/${TAG}_cold_call.json 2>&1
rc=$?; tail -c 600 gpurun_out/${TAG}_cold_call.json; [ $rc -lt 124 ] || exit $rc
echo done
