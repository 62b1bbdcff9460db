#!/bin/bash
# Round-5 A/B of the chunk-plan defaults (lib/variants/librt_base.so = the previous defaults)
# against the working build, in one process per workload: config 3 (10 000 spp), 1080p / 1000 spp
# (both streams), config 5 (1000 spp). Outputs gpurun_out/${TAG}_*.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05d}
V=$(ls ray-tracing-gpu-vulkan_amd/lib/variants/*.so)
run() { local name=$1; shift; timeout -k 10 500 python -u scripts/perf_variants.py "$@" $V > gpurun_out/${TAG}_$name.log 2>&1
        local rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_$name.log | tail -8; [ $rc -lt 124 ] || exit $rc; }
run c3_10000 --spp 10000 --rounds 2 --accels 2 --rng 2
run c3_1000 --spp 1000 --rounds 4 --accels 2 --rng 2,0
run c5_1000 --spp 1000 --rounds 3 --accels 2 --rng 2 --width 3840 --height 2160 --grid 158
timeout -k 10 300 python -u scripts/band_tune.py 8 10000 --rounds 3 --set default: > gpurun_out/${TAG}_band.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_band.log | tail -3; [ $rc -lt 124 ] || exit $rc
echo done
