#!/bin/bash
# Head / tail chunk split of the LPT order (RT_HEAD_CHUNKS, RT_TAIL_TILES_PM) on
# the GPU box: parity tests of the split, in-process frame-time A/B at config 3 (10 000 spp) and
# config 5, then the config 3 trace kernel's HBM traffic per head chunk count (rocprofv3 --pmc
# WRITE_SIZE / FETCH_SIZE, one pass each). Outputs gpurun_out/head/. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/head
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "head_tail or chunk_invariance or tail_steals or config3_hash" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
AB_RNG=hash timeout -k 10 300 python -u scripts/env_ab.py RT_HEAD_CHUNKS 10000 h25=25 h3=3 h6=6 h12=12 > $OUT/ab_head.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_head.log; [ $rc -eq 0 ] || exit $rc
AB_RNG=hash timeout -k 10 300 python -u scripts/env_ab.py RT_TAIL_TILES_PM 10000 t50=50 t100=100 t200=200 t1000=1000 > $OUT/ab_tail.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_tail.log; [ $rc -eq 0 ] || exit $rc
AB_RNG=hash AB_W=3840 AB_H=2160 AB_K=158 timeout -k 10 300 python -u scripts/env_ab.py RT_TAIL_TILES_PM 1000 t100=100 t1000=1000 > $OUT/ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_c5.log; [ $rc -eq 0 ] || exit $rc
for H in ${HEADS:-25 3}; do
    for CTR in WRITE_SIZE FETCH_SIZE; do
        RT_HEAD_CHUNKS=$H timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR --output-format csv \
            -d "$ROOT/$OUT/c${H}_$CTR" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --profile \
            > $OUT/c${H}_$CTR.log 2>&1 < /dev/null
        rc=$?; echo "head $H $CTR rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
done
python3 scripts/chunk_traffic.py $OUT ${HEADS:-25 3} | tee $OUT/summary.txt
