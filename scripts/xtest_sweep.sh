# The sample-split exchange on a one-rank NCCL group (--exchange-test) against the plain frame, at
# the N=8 per-rank share (12 spp), for 1-3 frames in flight.
set -e
for inf in 1 2 3; do
MASTER_ADDR=127.0.0.1 MASTER_PORT=2954$inf WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 200 python bench.py --exchange-test --no-cpu-baseline --no-brute-line --steps 40 --spp 12 --inflight $inf > gpurun_out/xt_${inf}_12.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-brute-line --steps 40 --spp 12 --inflight $inf > gpurun_out/st_${inf}_12.log 2>&1
done
