#!/bin/bash
# A/B session on the GPU box: parity gate on the working build, then in-process timing against the
# variant libraries under ray-tracing-gpu-vulkan_amd/lib/variants/ (config 3 at 1000 spp in both
# streams, config 5 at 100 spp). Outputs gpurun_out/ab_*.log. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "golden or vs_oracle or lattice or near_cull or chunk or treelet" > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
V=ray-tracing-gpu-vulkan_amd/lib/variants/*.so
timeout -k 10 300 python scripts/perf_variants.py --spp 1000 --rounds 3 --accels 2 --rng 2,0 $V > gpurun_out/ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/perf_variants.py --spp 100 --rounds 3 --accels 2 --rng 2 --width 3840 --height 2160 --grid 158 $V > gpurun_out/ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_c5.log; exit $rc
