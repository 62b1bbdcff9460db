#!/bin/bash
# Round profile on the GPU box (outputs under gpurun_out/round/): rocprofv3 kernel-trace stats of
# the bench command (one frame in flight, so each launch runs alone and its duration is the
# kernel's), then one --pmc pass per line of scripts/pmc_quick.txt (kernel-trace only
# beside --pmc), then the JSON summaries bench.py reads (profiles/pmc_traffic.json,
# profiles/pmc_valu.json, written in the gpurun_out copy and merged back by the caller).
# Stops at the first fault-like exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
mkdir -p "$OUT"
export TMPDIR=/tmp
BARGS=${BENCH_ARGS:-"--steps 20 --warmup 2 --profile --inflight 1"}   # 22 launches: the first (no LPT order yet) barely moves the average
PARGS=${PMC_BENCH_ARGS:-"--steps 2 --warmup 1 --profile --inflight 1"}
KEY=${KEY:-lbvh-1920x1080-100spp-grid11-n1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 bench.py $BARGS > "$OUT/stats.log" 2>&1
rc=$?; echo "stats rc=$rc"; tail -1 "$OUT/stats.log"
[ $rc -eq 0 ] || exit $rc
i=0
while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line --output-format csv -d "$OUT/p$i" -o run -- \
        python3 bench.py $PARGS > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i ($line) rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done < scripts/pmc_quick.txt
mkdir -p gpurun_out/profiles_new
cp profiles/pmc_traffic.json profiles/pmc_valu.json gpurun_out/profiles_new/ 2>/dev/null
python3 scripts/pmc_to_json.py "$KEY" "$OUT/p1" gpurun_out/profiles_new/pmc_valu.json
python3 scripts/traffic_from_pmc.py "$KEY" "$OUT/p3" "$OUT/p4" gpurun_out/profiles_new/pmc_traffic.json
python3 scripts/pmc_summary.py "$OUT/p1" "$OUT/p2" > "$OUT/sq_summary.txt"
echo done
