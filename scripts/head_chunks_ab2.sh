#!/bin/bash
# Head / tail chunk split, second pass (cost normalisation in the LPT order): parity tests, then
# interleaved A/B of split settings on the config 3 frame (10 000 spp) and config 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/head2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "head_tail or chunk_invariance or tail_steals or config3_hash" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/envs_ab.py 10000 8 none=RT_TAIL_TILES_PM:1000 h3t100=RT_HEAD_CHUNKS:3 \
    h3t200=RT_HEAD_CHUNKS:3,RT_TAIL_TILES_PM:200 h6t100=RT_HEAD_CHUNKS:6 h4t150=RT_HEAD_CHUNKS:4,RT_TAIL_TILES_PM:150 \
    > $OUT/ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_c3.log; [ $rc -eq 0 ] || exit $rc
AB_W=3840 AB_H=2160 AB_K=158 timeout -k 10 300 python -u scripts/envs_ab.py 1000 6 none=RT_TAIL_TILES_PM:1000 \
    h1t100=RT_HEAD_CHUNKS:1 h1t200=RT_HEAD_CHUNKS:1,RT_TAIL_TILES_PM:200 > $OUT/ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_c5.log; exit $rc
