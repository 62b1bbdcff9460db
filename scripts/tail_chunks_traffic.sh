#!/bin/bash
# Tail chunk count of the head / tail split: config 3 trace-kernel WRITE_SIZE (rocprofv3 --pmc, the
# bench's LPT-ordered frames) and an interleaved frame-time A/B. Outputs gpurun_out/tailc/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/tailc
mkdir -p $OUT
IFS=";" read -ra SETL <<< "${SETS:-12 3 150;12 3 200;16 3 150}"
for S in "${SETL[@]}"; do
    set -- $S
    RT_SAMPLE_CHUNKS=$1 RT_HEAD_CHUNKS=$2 RT_TAIL_TILES_PM=$3 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE \
        --output-format csv -d "$ROOT/$OUT/c$1_h$2_t$3" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --profile \
        > $OUT/c$1_h$2_t$3.log 2>&1 < /dev/null
    rc=$?; echo "tail chunks $1 head $2 tail $3 per mille rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY' | tee $OUT/summary.txt
import glob, sys
sys.path.insert(0, "scripts")
from pmc_collect import dispatches
for d in sorted(glob.glob("gpurun_out/tailc/c*_h*_t*/")):
    ds = dispatches(d.rstrip("/"))
    print(d.split("/")[-2] + ": " + ", ".join(f"{e['WRITE_SIZE'] * 1024 / 1e9:.3f} GB / {e['dur_ns'] / 1e6:.1f} ms" for e in ds))
PY
AB=${AB:-"default=RT_TAIL_TILES_PM:- c12t150=RT_SAMPLE_CHUNKS:12,RT_HEAD_CHUNKS:3,RT_TAIL_TILES_PM:150 c12t200=RT_SAMPLE_CHUNKS:12,RT_HEAD_CHUNKS:3 c16t150=RT_SAMPLE_CHUNKS:16,RT_HEAD_CHUNKS:3,RT_TAIL_TILES_PM:150"}
timeout -k 10 500 python -u scripts/envs_ab.py 10000 10 $AB > $OUT/ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_c3.log; exit $rc
