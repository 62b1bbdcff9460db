#!/bin/bash
# One process per (path, library) of scripts/c5_gap_probe.py --solo: each with bench.py's own
# streams, so each sees the hardware-queue assignment the bench would. Output: gpurun_out/$TAG_*.
set -o pipefail
TAG=${TAG:-gap}
SPP=${SPP:-1000}
FRAMES=${FRAMES:-5}
mkdir -p gpurun_out
for lib in "$@"; do
  for path in single multi; do
    n=$(basename "$lib" .so)
    timeout -k 10 120 python -u scripts/c5_gap_probe.py --solo "$path" "$lib" --spp "$SPP" --frames "$FRAMES" \
      --rounds 1 > "gpurun_out/${TAG}_${path}_${n}.log" 2>&1 || { echo "FAILED $path $lib"; exit 1; }
    grep '"ms_per_step"' "gpurun_out/${TAG}_${path}_${n}.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print('$path', d['lib'], d['ms_per_step'], d['kernel_ms'], d['overhead_ms'])"
  done
done
