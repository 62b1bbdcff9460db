#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in 0 8; do
  BENCH_ARGS="--steps 1 --warmup 0 --profile --spp 16 --compact $c" PMC_FILE=scripts/pmc_compare.txt bash scripts/gpu_pmc.sh > /dev/null 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
  mv gpurun_out/pmc gpurun_out/pmc_c$c
done
echo ok
