#!/bin/bash
# HBM traffic of the config 3 trace kernel against the sample-chunk count (RT_SAMPLE_CHUNKS): one
# rocprofv3 --pmc pass for WRITE_SIZE and one for FETCH_SIZE per count (each its own run), then
# scripts/chunk_traffic.py prints GB per launch and the kernel time. Outputs gpurun_out/chunks/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/chunks
mkdir -p $OUT
for C in ${CHUNKS:-25 8 3}; do
    for CTR in WRITE_SIZE FETCH_SIZE; do
        RT_SAMPLE_CHUNKS=$C timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR --output-format csv \
            -d "$ROOT/$OUT/c${C}_$CTR" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --profile \
            > $OUT/c${C}_$CTR.log 2>&1 < /dev/null
        rc=$?; echo "chunks $C $CTR rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
done
python3 scripts/chunk_traffic.py $OUT ${CHUNKS:-25 8 3} | tee $OUT/summary.txt
