#!/bin/bash
# Round-6 A/B session 3: wave priority (s_setprio) raised to RT_WALK_PRIO around the segment walk
# and / or to RT_REFILL_PRIO around the unit refill, against the shipped build (perf_variants: config 3 at
# 1 000 spp in both streams, config 5 at 100 spp). Outputs gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06q}
VARIANTS=${VARIANTS:-$(ls ray-tracing-gpu-vulkan_amd/lib/variants/*.so)}

C5="--width 3840 --height 2160 --grid 158"
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
timeout -k 10 500 python -u scripts/perf_variants.py --spp 1000 --rounds ${ROUNDS:-5} --accels 2 --rng 2,0 $VARIANTS > gpurun_out/${TAG}_ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c3.log | tail -12; fatal $rc ab_c3
timeout -k 10 400 python -u scripts/perf_variants.py --spp 100 --rounds ${ROUNDS:-5} --accels 2 --rng 2 $C5 $VARIANTS > gpurun_out/${TAG}_ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c5.log | tail -6; fatal $rc ab_c5
echo done
