#!/bin/bash
# Round-5: lane utilisation (RT_UTIL builds) and one SQ PMC pass per library variant on config 3
# at 100 spp (scripts/frame_once.py), then a second launch-plan sweep of the N = 8 band and of the
# whole frame. Outputs gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05c}
VD=ray-tracing-gpu-vulkan_amd/lib/variants
for u in util util_specmerged; do
    [ -f $VD/librt_$u.so ] || continue
    RT_LIB=$VD/librt_$u.so RT_WALK=0 timeout -k 10 120 python -u scripts/lane_util.py 100 > gpurun_out/${TAG}_lane_$u.log 2>&1
    rc=$?; echo "lane $u rc=$rc"; tail -25 gpurun_out/${TAG}_lane_$u.log; [ $rc -lt 124 ] || exit $rc
done
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
for lib in ray-tracing-gpu-vulkan_amd/lib/librt_mi355x.so $VD/librt_specmerged.so; do
    name=$(basename "$lib" .so)
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d "$(pwd)/gpurun_out/${TAG}_pmc/$name" -o run -- \
        python3 scripts/frame_once.py "$lib" 100 > gpurun_out/${TAG}_pmc_$name.log 2>&1 < /dev/null
    rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_pmc_$name.log; exit $rc; }
    python3 scripts/pmc_summary.py "gpurun_out/${TAG}_pmc/$name" > gpurun_out/${TAG}_pmc_${name}_summary.txt 2>&1
    grep -v "true>" gpurun_out/${TAG}_pmc_${name}_summary.txt | head -20
done
if [ "${SKIP_BAND:-0}" != 1 ]; then
timeout -k 10 300 python -u scripts/band_tune.py 8 10000 --rounds 3 --set default: tail300:tail_tiles_pm=300 tail400:tail_tiles_pm=400 tail500:tail_tiles_pm=500 min128_tail300:unit_min_samples=128,tail_tiles_pm=300 min128_tail400:unit_min_samples=128,tail_tiles_pm=400 min64_tail400:unit_min_samples=64,tail_tiles_pm=400 > gpurun_out/${TAG}_band_tune.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_band_tune.log | tail -9; [ $rc -lt 124 ] || exit $rc
timeout -k 10 300 python -u scripts/band_tune.py 1 10000 --full --rounds 3 --set default: tail300:tail_tiles_pm=300 tail400:tail_tiles_pm=400 min128_tail300:unit_min_samples=128,tail_tiles_pm=300 > gpurun_out/${TAG}_full_tune.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_full_tune.log | tail -6; [ $rc -lt 124 ] || exit $rc
fi
echo done
