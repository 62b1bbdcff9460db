#!/bin/bash
# Round 4: the wave-wide candidate queue (walk form 16) — parity (the full -m gpu suite runs it in
# every FORMS test), in-process A/B against the default walk (config 3, 1000 spp, both streams),
# lane utilisation per code point (RT_UTIL build), and the config 5 multi-path step overhead.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04b}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
V=$(ls ray-tracing-gpu-vulkan_amd/lib/variants/*.so 2>/dev/null | grep -v util)
timeout -k 10 400 python scripts/perf_variants.py --spp 1000 --rounds 4 --accels 2 --rng 2,0 --walk 0,16 $V > gpurun_out/${TAG}_ab_cq.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_cq.log; fatal $rc ab_cq
timeout -k 10 400 python scripts/perf_variants.py --spp 100 --rounds 4 --accels 2 --rng 2 --width 3840 --height 2160 --grid 158 $V > gpurun_out/${TAG}_ab_c5.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c5.log; fatal $rc ab_c5
for w in 0 16; do
  RT_LIB=ray-tracing-gpu-vulkan_amd/lib/variants/librt_util.so RT_WALK=$w timeout -k 10 200 python scripts/lane_util.py 100 > gpurun_out/${TAG}_util_walk$w.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_util_walk$w.log; fatal $rc util$w
done
timeout -k 10 300 python bench.py --config 5 --path multi --gpus 1 --steps 3 --warmup 2 --no-cpu-baseline --no-rebuild-check > gpurun_out/${TAG}_bench_c5_multi.json 2> gpurun_out/${TAG}_bench_c5_multi.err
rc=$?; tail -c 300 gpurun_out/${TAG}_bench_c5_multi.json; fatal $rc bench_c5_multi
RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --spp 1000 \
    > gpurun_out/${TAG}_rehearsal_n2_gloo.json 2> gpurun_out/${TAG}_rehearsal_n2_gloo.err
rc=$?; echo "gloo n2 rc=$rc"; tail -c 600 gpurun_out/${TAG}_rehearsal_n2_gloo.json; fatal $rc gloo_n2
timeout -k 10 300 python bench.py --path multi --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-rebuild-check \
    > gpurun_out/${TAG}_bench_multi_n1.json 2> gpurun_out/${TAG}_bench_multi_n1.err
rc=$?; echo "multi n1 rc=$rc"; tail -c 400 gpurun_out/${TAG}_bench_multi_n1.json; fatal $rc multi_n1
echo done
