#!/bin/bash
# PMC A/B of library variants: same bench command, one SQ pass per library.
# usage: gpu_pmc_ab.sh lib1.so lib2.so ...   (BENCH_ARGS, PMC overridable)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
BARGS=${BENCH_ARGS:-"--steps 1 --warmup 0 --profile --spp 16"}
PMC=${PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"}
for lib in "$@"; do
    name=$(basename "$lib" .so)
    RT_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --pmc $PMC --output-format csv \
        -d "gpurun_out/pmcab/$name" -o run -- python3 bench.py $BARGS > "gpurun_out/pmcab_$name.log" 2>&1
    rc=$?; echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "gpurun_out/pmcab_$name.log"; exit $rc; fi
done
for lib in "$@"; do python3 scripts/pmc_summary.py "gpurun_out/pmcab/$(basename "$lib" .so)" | grep -v "true>" | grep -A12 "false>" | head -13; done
