#!/bin/bash
# Round profile on the GPU box (outputs under gpurun_out/round${TAG}/): rocprofv3 kernel-trace stats
# of the bench command (one frame in flight, so each launch runs alone and its duration is the
# kernel's), then one --pmc pass per line of scripts/pmc_quick.txt (kernel-trace only beside
# --pmc, each pass its own run), then scripts/pmc_collect.py writes the workload's record into
# gpurun_out/profiles_new/pmc.json (stamped with the library's sha256; copy it to profiles/).
# CONFIG=3 (default) or 5 selects the BASELINE config. Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=${CONFIG:-3}
OUT=gpurun_out/round${TAG:-}_c${CONFIG}
mkdir -p "$OUT" gpurun_out/profiles_new
export TMPDIR=/tmp
ROOT=$(pwd)
if [ "$CONFIG" = 5 ]; then
    BARGS=${BENCH_ARGS:-"--config 5 --steps 2 --warmup 2 --profile"}
    PARGS=${PMC_BENCH_ARGS:-"--config 5 --steps 1 --warmup 2 --profile"}
    KEY=${KEY:-lbvh-hash-3840x2160-1000spp-grid158-n1}
else
    BARGS=${BENCH_ARGS:-"--steps 3 --warmup 2 --profile"}
    PARGS=${PMC_BENCH_ARGS:-"--steps 1 --warmup 2 --profile"}
    KEY=${KEY:-lbvh-hash-1920x1080-10000spp-grid11-n1}
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" $BARGS > "$OUT/stats.log" 2>&1 < /dev/null
rc=$?; echo "stats rc=$rc"; tail -c 300 "$OUT/stats.log"; echo
[ $rc -eq 0 ] || exit $rc
i=0
while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $line --output-format csv -d "$ROOT/$OUT/p$i" -o run -- \
        python3 "$ROOT/bench.py" $PARGS > "$OUT/p$i.log" 2>&1 < /dev/null
    rc=$?; echo "pass $i ($line) rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done < scripts/pmc_quick.txt
[ -f gpurun_out/profiles_new/pmc.json ] || cp profiles/pmc.json gpurun_out/profiles_new/pmc.json 2>/dev/null
python3 scripts/pmc_collect.py "$KEY" ray-tracing-gpu-vulkan_amd/lib/librt_mi355x.so "$OUT/p1" "$OUT/p3" "$OUT/p4" "$OUT/p2" \
    --tcc "$OUT/p5" gpurun_out/profiles_new/pmc.json
python3 scripts/pmc_summary.py "$OUT/p1" "$OUT/p2" > "$OUT/sq_summary.txt" 2>&1
echo done
