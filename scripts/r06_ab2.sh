#!/bin/bash
# Round-6 A/B session 2: the single-loop grid walk with one latch (librt_single.so) against the
# shipped build (perf_variants: config 3 at 1 000 spp in both streams, config 5 at 100 spp) and its
# lane utilisation (RT_UTIL), then the tail launch plan (unit_min_samples, tail_tiles_pm,
# sample_chunks) on the N = 8 bands of configs 4 / 5 and the whole frames of configs 3 / 5, more
# interleaved rounds (scripts/band_tune.py). Outputs gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06d}
V=ray-tracing-gpu-vulkan_amd/lib/variants
C5="--width 3840 --height 2160 --grid 158"
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ "${SKIP_WALK:-0}" != 1 ]; then
timeout -k 10 400 python -u scripts/perf_variants.py --spp 1000 --rounds 3 --accels 2 --rng 2,0 $V/librt_single.so > gpurun_out/${TAG}_ab_single_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_single_c3.log | tail -4; fatal $rc ab_c3
timeout -k 10 300 python -u scripts/perf_variants.py --spp 100 --rounds 3 --accels 2 --rng 2 $C5 $V/librt_single.so > gpurun_out/${TAG}_ab_single_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_single_c5.log | tail -2; fatal $rc ab_c5
RT_LIB=$V/librt_util_single.so timeout -k 10 200 python -u scripts/lane_util.py 100 > gpurun_out/${TAG}_lane_util_single.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_lane_util_single.log | tail -16; fatal $rc lane_util
fi
run() { name=$1; shift; timeout -k 10 400 python scripts/band_tune.py "$@" > gpurun_out/${TAG}_$name.log 2>&1
        rc=$?; echo "== $name"; grep -v "amdgpu.ids\|^{" gpurun_out/${TAG}_$name.log; fatal $rc $name; }
SETS="default: min32:unit_min_samples=32 t400:tail_tiles_pm=400 min32_t400:unit_min_samples=32,tail_tiles_pm=400"
run tune2_c5_band5 8 1000 $C5 --rank 5 --rounds 5 --set $SETS
run tune2_c5_band0 8 1000 $C5 --rank 0 --rounds 5 --set $SETS
run tune2_c3_band0 8 10000 --rank 0 --rounds 5 --set $SETS
run tune2_c3_band7 8 10000 --rank 7 --rounds 5 --set $SETS
run tune2_c3_full 1 10000 --full --rounds 3 --set default: t400:tail_tiles_pm=400 min32_t400:unit_min_samples=32,tail_tiles_pm=400
run tune2_c5_full 1 1000 $C5 --full --rounds 4 --set default: tail6:sample_chunks=6 t400:tail_tiles_pm=400 tail6_t400:sample_chunks=6,tail_tiles_pm=400
echo done
