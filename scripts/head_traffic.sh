#!/bin/bash
# Config 3 trace-kernel HBM traffic with and without the head / tail chunk split (rocprofv3 --pmc
# WRITE_SIZE / FETCH_SIZE, one pass each; the bench's timed frame is the LPT-ordered one), plus an
# interleaved frame-time A/B. Outputs gpurun_out/headt/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/headt
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "head_tail or chunk_invariance or tail_steals or config3_hash or lpt" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for T in 200 1000; do
    for CTR in WRITE_SIZE FETCH_SIZE; do
        RT_TAIL_TILES_PM=$T timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR --output-format csv \
            -d "$ROOT/$OUT/c${T}_$CTR" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --profile \
            > $OUT/c${T}_$CTR.log 2>&1 < /dev/null
        rc=$?; echo "tail $T $CTR rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
done
python3 - <<'PY' | tee $OUT/summary.txt
import sys
sys.path.insert(0, "scripts")
from pmc_collect import dispatches
for t in (200, 1000):
    for ctr in ("WRITE_SIZE", "FETCH_SIZE"):
        ds = dispatches(f"gpurun_out/headt/c{t}_{ctr}")
        print(f"tail {t} per mille, {ctr}: " + ", ".join(f"{e[ctr] * 1024 / 1e9:.3f} GB / {e['dur_ns'] / 1e6:.1f} ms" for e in ds))
PY
timeout -k 10 400 python -u scripts/envs_ab.py 10000 8 nohead=RT_TAIL_TILES_PM:1000 default=RT_TAIL_TILES_PM:- > $OUT/ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_c3.log; exit $rc
