#!/bin/bash
# Config 5 (4K, 1000 spp, 99 860 spheres) in-process A/B of the working build against
# lib/variants/*.so at the library's chunk count and forced counts (CHUNKS5). gpurun_out/steal_c5k_*.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=ray-tracing-gpu-vulkan_amd/lib/variants/*.so
for C in ${CHUNKS5:-default 2 1}; do
    if [ "$C" = default ]; then E=""; else E="RT_SAMPLE_CHUNKS=$C"; fi
    env $E timeout -k 10 300 python scripts/perf_variants.py --rounds 3 --accels 2 --rng 2 --spp 1000 --width 3840 \
        --height 2160 --grid 158 $V > gpurun_out/steal_c5k_$C.log 2>&1 || exit 1
    echo "c5 1000spp chunks=$C"; grep -v amdgpu.ids gpurun_out/steal_c5k_$C.log
done
