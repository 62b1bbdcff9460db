#!/bin/bash
# Round-6 A/B session: the single-loop grid walk (librt_single.so, -DRT_GRID_SINGLE) and the
# texel-major fixed-point sums (librt_aos.so, -DRT_FIXED_AOS) against the shipped build in one
# process (scripts/perf_variants.py: config 3 at 1 000 spp in both streams, config 5 at 100 spp;
# every variant image bit-equal), the lane utilisation of both walks (RT_UTIL builds,
# scripts/lane_util.py) and one rocprofv3 WRITE_SIZE pass per fixed-point layout (config 3 frame at
# 1 000 spp, scripts/frame_once.py). Outputs gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06c}
V=ray-tracing-gpu-vulkan_amd/lib/variants
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
timeout -k 10 400 python -u scripts/perf_variants.py --spp 1000 --rounds 3 --accels 2 --rng 2,0 $V/librt_single.so $V/librt_aos.so > gpurun_out/${TAG}_ab_single_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_single_c3.log | tail -8; fatal $rc ab_c3
timeout -k 10 300 python -u scripts/perf_variants.py --spp 100 --rounds 3 --accels 2 --rng 2 --width 3840 --height 2160 --grid 158 $V/librt_single.so $V/librt_aos.so > gpurun_out/${TAG}_ab_single_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_single_c5.log | tail -6; fatal $rc ab_c5
for L in util util_single; do
RT_LIB=$V/librt_$L.so timeout -k 10 200 python -u scripts/lane_util.py 100 > gpurun_out/${TAG}_lane_util_$L.log 2>&1
rc=$?; echo "== $L"; grep -v amdgpu.ids gpurun_out/${TAG}_lane_util_$L.log | tail -16; fatal $rc lane_util_$L
done
export TMPDIR=/tmp
for L in default aos; do
    LIB=$V/librt_$L.so; [ $L = default ] && LIB=ray-tracing-gpu-vulkan_amd/lib/librt_mi355x.so
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$(pwd)/gpurun_out/${TAG}_ws_$L" -o run -- \
        python3 scripts/frame_once.py $LIB 1000 > gpurun_out/${TAG}_ws_$L.log 2>&1 < /dev/null
    rc=$?; echo "write_size $L rc=$rc"; fatal $rc ws_$L
done
python3 scripts/pmc_traffic.py gpurun_out/${TAG}_ws_default gpurun_out/${TAG}_ws_aos | grep -i trace
echo done
