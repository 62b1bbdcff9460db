#!/bin/bash
# GPU-box session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a test failure (exit 1) lets later steps run, any
# fault / abort / segfault / timeout (anything else non-zero) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
nproc > "$OUT/nproc.txt"; lscpu | grep -i "model name" >> "$OUT/nproc.txt"
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest_gpu 600 python -m pytest tests -m gpu -q -rf --maxfail=20
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py --steps 5 --warmup 2
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 3 --warmup 1 --profile
fi
echo done
