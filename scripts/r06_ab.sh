#!/bin/bash
# Round-6 A/B session: the single-loop grid walk (librt_single.so, -DRT_GRID_SINGLE) against the
# shipped build in one process (scripts/perf_variants.py: config 3 at 1 000 spp in both streams,
# config 5 at 100 spp; every variant image bit-equal), and the lane utilisation of both walks
# (RT_UTIL builds, scripts/lane_util.py). Outputs gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06c}
V=ray-tracing-gpu-vulkan_amd/lib/variants
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
timeout -k 10 400 python -u scripts/perf_variants.py --spp 1000 --rounds 3 --accels 2 --rng 2,0 $V/librt_single.so > gpurun_out/${TAG}_ab_single_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_single_c3.log | tail -8; fatal $rc ab_c3
timeout -k 10 300 python -u scripts/perf_variants.py --spp 100 --rounds 3 --accels 2 --rng 2 --width 3840 --height 2160 --grid 158 $V/librt_single.so > gpurun_out/${TAG}_ab_single_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_single_c5.log | tail -6; fatal $rc ab_c5
for L in util util_single; do
RT_LIB=$V/librt_$L.so timeout -k 10 200 python -u scripts/lane_util.py 100 > gpurun_out/${TAG}_lane_util_$L.log 2>&1
rc=$?; echo "== $L"; grep -v amdgpu.ids gpurun_out/${TAG}_lane_util_$L.log | tail -16; fatal $rc lane_util_$L
done
echo done
