#!/bin/bash
# Round-6 launch-plan A/B for the N = 8 bands (the per-band tail after the work queue runs dry):
# unit_min_samples / tail_tiles_pm / sample_chunks on one rank's band of configs 4 and 5 and on
# the whole config 5 frame, interleaved rounds in one process (scripts/band_tune.py). Outputs
# gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06b}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest
fi
C5="--width 3840 --height 2160 --grid 158"
timeout -k 10 300 python scripts/band_tune.py 8 1000 $C5 --rank 5 --rounds 3 --set default: min64:unit_min_samples=64 \
    min32:unit_min_samples=32 min16:unit_min_samples=16 min32_t400:unit_min_samples=32,tail_tiles_pm=400 \
    min32_t200:unit_min_samples=32,tail_tiles_pm=200 > gpurun_out/${TAG}_tune_c5_band.log 2>&1
rc=$?; head -8 gpurun_out/${TAG}_tune_c5_band.log; fatal $rc tune_c5_band
timeout -k 10 300 python scripts/band_tune.py 8 10000 --rank 0 --rounds 3 --set default: min96:unit_min_samples=96 \
    min64:unit_min_samples=64 min48:unit_min_samples=48 min64_t400:unit_min_samples=64,tail_tiles_pm=400 \
    > gpurun_out/${TAG}_tune_c3_band.log 2>&1
rc=$?; head -7 gpurun_out/${TAG}_tune_c3_band.log; fatal $rc tune_c3_band
timeout -k 10 300 python scripts/band_tune.py 1 1000 $C5 --full --rounds 3 --set default: tail6:sample_chunks=6 \
    tail10:sample_chunks=10 min32:unit_min_samples=32 head2:head_chunks=2 > gpurun_out/${TAG}_tune_c5_full.log 2>&1
rc=$?; head -7 gpurun_out/${TAG}_tune_c5_full.log; fatal $rc tune_c5_full
echo done
