# Full round evidence on one GPU: parity tests, rocprofv3 stats + PMC passes, bench lines
# (default N=1 workload, BASELINE configs 3 and 5), an N=2 sample-split rehearsal. Stops at the
# first failure.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
bash scripts/round_profile.sh > gpurun_out/round_profile.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1
timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-brute-line > gpurun_out/bench_c3.log 2>&1
timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-brute-line > gpurun_out/bench_c5.log 2>&1
RT_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2_split.log 2>&1
