#!/bin/bash
# Round profile: kernel-trace stats of the bench command, then separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ) over the same command. Outputs under gpurun_out/profile/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/profile
mkdir -p "$OUT"
export TMPDIR=/tmp
BARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --profile"}
run() {  # run NAME CMD...
    local name=$1; shift
    timeout -k 10 600 "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
run stats rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $BARGS
run fetch rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $BARGS
run write rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $BARGS
run sq rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d "$OUT/sq" -o run -- python3 bench.py $BARGS
echo done
