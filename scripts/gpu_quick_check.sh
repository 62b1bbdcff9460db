set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench1.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-brute-line --spp 12 --steps 20 > gpurun_out/bench_spp12.log 2>&1
