#!/bin/bash
# In-process A/B of the variant libraries under ray-tracing-gpu-vulkan_amd/lib/variants/ against the
# working build (images must be bit-identical): config 3 at 1000 spp in both streams, config 5 at
# 100 spp. Outputs gpurun_out/${TAG}_ab_*.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04}
V=$(ls ray-tracing-gpu-vulkan_amd/lib/variants/*.so)
timeout -k 10 400 python scripts/perf_variants.py --spp 1000 --rounds ${ROUNDS:-4} --accels 2 --rng 2,0 $V > gpurun_out/${TAG}_ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c3.log; [ $rc -lt 124 ] || exit $rc
timeout -k 10 400 python scripts/perf_variants.py --spp 100 --rounds ${ROUNDS:-4} --accels 2 --rng 2 --width 3840 --height 2160 --grid 158 $V > gpurun_out/${TAG}_ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c5.log; exit $rc
