# Tile isolation (RT_ISOLATE_TILES) with two frames in flight, bench frames at 100 and 12 spp.
set -e
for iso in 0 32 64; do for s in 100 12; do
RT_ISOLATE_TILES=$iso timeout -k 10 200 python bench.py --no-cpu-baseline --no-brute-line --steps 30 --spp $s > gpurun_out/iso_${iso}_$s.log 2>&1
done; done
