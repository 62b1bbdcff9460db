# Quick GPU check: parity tests, the default bench line, a 12-spp line (the N=8 per-rank share),
# the RCCL exchange path on a one-rank NCCL group, an N=2 sample-split rehearsal (gloo, shared GPU).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench1.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-brute-line --spp 12 --steps 30 > gpurun_out/bench_spp12.log 2>&1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 300 python bench.py --exchange-test --no-cpu-baseline --no-brute-line --steps 10 > gpurun_out/bench_xtest.log 2>&1
RT_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2_split.log 2>&1
