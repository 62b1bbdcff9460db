set -e
for inf in 1 2; do for s in 100 12; do
MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$inf WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 200 python bench.py --exchange-test --no-cpu-baseline --no-brute-line --steps 20 --spp $s --inflight $inf > gpurun_out/xt_${inf}_$s.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-brute-line --steps 20 --spp $s --inflight $inf > gpurun_out/st_${inf}_$s.log 2>&1
done; done
