#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only beside --pmc, no
# sys/runtime traces) over a short bench run. Stops at the first fault-like exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 0 --profile"}
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    echo "== pass $i: $line"
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line --output-format csv -d "$OUT/p$i" -o run -- \
        python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"; tail -2 "$OUT/p$i.log"
    if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
        echo "stopping (rc=$rc)"; exit $rc
    fi
done < "${PMC_FILE:-scripts/pmc_passes.txt}"
echo done
