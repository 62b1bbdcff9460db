#!/bin/bash
# Round-5 A/B on the GPU box: the variant libraries under ray-tracing-gpu-vulkan_amd/lib/variants/
# against the working build in one process (images bit-identical): config 3 at 1000 spp in both
# streams, config 5 at 100 spp; then the launch-plan sweep of config 4's N = 8 band (band_tune.py).
# Outputs gpurun_out/${TAG}_*.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05b}
V=$(ls ray-tracing-gpu-vulkan_amd/lib/variants/*.so)
if [ "${SKIP_AB:-0}" != 1 ]; then
timeout -k 10 500 python -u scripts/perf_variants.py --spp 1000 --rounds ${ROUNDS:-4} --accels 2 --rng 2,0 $V > gpurun_out/${TAG}_ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c3.log | tail -30; [ $rc -lt 124 ] || exit $rc
timeout -k 10 400 python -u scripts/perf_variants.py --spp 100 --rounds ${ROUNDS:-4} --accels 2 --rng 2 --width 3840 --height 2160 --grid 158 $V > gpurun_out/${TAG}_ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c5.log | tail -20; [ $rc -lt 124 ] || exit $rc
fi
if [ "${SKIP_BAND:-0}" != 1 ]; then
timeout -k 10 300 python -u scripts/band_tune.py 8 10000 --rounds 3 > gpurun_out/${TAG}_band_tune.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_band_tune.log | tail -12; [ $rc -lt 124 ] || exit $rc
fi
echo done
