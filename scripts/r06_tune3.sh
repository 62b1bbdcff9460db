#!/bin/bash
# Round-6 tail sweep on config 4's N = 8 band (rank 0, 135 rows, 10 000 spp) and config 5's band:
# forced tail chunk counts, head chunks, tail tile share and the one-by-one hand-out reserve,
# interleaved rounds in one process (scripts/band_tune.py). Outputs gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06h}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest
fi
run() { name=$1; shift; timeout -k 10 500 python scripts/band_tune.py "$@" > gpurun_out/${TAG}_$name.log 2>&1
        rc=$?; echo "== $name"; grep -v "amdgpu.ids\|^{" gpurun_out/${TAG}_$name.log; fatal $rc $name; }
run c3_band0 8 10000 --rank 0 --rounds 4 --set default: tail100:sample_chunks=100 tail150:sample_chunks=150 \
    head10:head_chunks=10 head30:head_chunks=30 t500:tail_tiles_pm=500 res0:refill_reserve=0 res32k:refill_reserve=32768
run c5_band5 8 1000 --width 3840 --height 2160 --grid 158 --rank 5 --rounds 4 --set default: tail25:sample_chunks=25 \
    tail40:sample_chunks=40 head3:head_chunks=3 t500:tail_tiles_pm=500 res0:refill_reserve=0 res32k:refill_reserve=32768
echo done
