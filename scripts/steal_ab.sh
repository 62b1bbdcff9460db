#!/bin/bash
# Tail-stealing / chunk-count A/B on the GPU box: parity gate, then the working build against
# lib/variants/*.so at the library's chunk count and at forced counts (RT_SAMPLE_CHUNKS):
# config 3 (1080p, SPP3 spp, CHUNKS) and config 5 (4K, 100 spp, CHUNKS5). Outputs
# gpurun_out/steal_*.log. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "golden or vs_oracle or lattice or near_cull or chunk or treelet" > gpurun_out/steal_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/steal_pytest.log; [ $rc -eq 0 ] || exit $rc
V=ray-tracing-gpu-vulkan_amd/lib/variants/*.so
run() {   # config tag, chunk setting, perf_variants args...
    local cfg=$1 C=$2; shift 2
    if [ "$C" = default ]; then E=""; else E="RT_SAMPLE_CHUNKS=$C"; fi
    env $E timeout -k 10 300 python scripts/perf_variants.py --rounds 3 --accels 2 --rng 2 "$@" $V > gpurun_out/steal_${cfg}_$C.log 2>&1
    local rc=$?; echo "$cfg chunks=$C"; grep -v amdgpu.ids gpurun_out/steal_${cfg}_$C.log; return $rc
}
for C in ${CHUNKS:-default 4 8}; do run c3 $C --spp ${SPP3:-1000} || exit 1; done
for C in ${CHUNKS5:-default}; do run c5 $C --spp 100 --width 3840 --height 2160 --grid 158 || exit 1; done
