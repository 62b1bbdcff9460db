#!/bin/bash
# WRITE_SIZE and FETCH_SIZE passes (one counter per run) over config 4's rank-0 band at the shipped
# build; summary in gpurun_out/${TAG}_band_pmc.json (scripts/band_pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05u}
for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$(pwd)/gpurun_out/${TAG}_band_pmc_$c" -o run -- \
        python3 scripts/band_probe.py 8 10000 --ranks 0 --reps 1 --no-full > gpurun_out/${TAG}_band_pmc_$c.log 2>&1 < /dev/null
    rc=$?; tail -c 200 gpurun_out/${TAG}_band_pmc_$c.log; [ $rc -eq 0 ] || { echo "pass $c rc=$rc"; exit $rc; }
done
python3 scripts/band_pmc_summary.py gpurun_out/${TAG}_band_pmc.json gpurun_out/${TAG}_band_pmc_WRITE_SIZE gpurun_out/${TAG}_band_pmc_FETCH_SIZE
