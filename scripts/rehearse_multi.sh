#!/bin/bash
# N > 1 rehearsal on a one-GPU box (outputs under gpurun_out/): the per-process bench path with 2
# ranks sharing the GPU over gloo (bands staged through host memory: a code-path test, never a
# reported number), then the rt_multi (C-ABI, one process) path at N = 1 on the full config 3
# frame, to compare with the single-GPU line. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --spp 1000 \
    > gpurun_out/rehearsal_n2_gloo.json 2> gpurun_out/rehearsal_n2_gloo.err
rc=$?; echo "gloo n2 rc=$rc"; tail -c 1500 gpurun_out/rehearsal_n2_gloo.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --path multi --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_multi_n1.json 2> gpurun_out/bench_multi_n1.err
rc=$?; echo "multi n1 rc=$rc"; tail -c 1500 gpurun_out/bench_multi_n1.json; exit $rc
