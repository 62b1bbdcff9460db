set -u
V=ray-tracing-gpu-vulkan_amd/lib/variants/*.so
timeout -k 10 300 python -u scripts/perf_variants.py --spp 1000 --rounds 3 --accels 2 --rng 2,0 $V > gpurun_out/ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/perf_variants.py --spp 100 --rounds 3 --accels 2 --rng 2 --width 3840 --height 2160 --grid 158 $V > gpurun_out/ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_c5.log; exit $rc
