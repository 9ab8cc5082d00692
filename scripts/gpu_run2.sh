#!/bin/bash
# GPU call: parity tests, default bench, nt-load A/B, rocprof stats + HBM counters
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
step nt_c1500 300 env PPTK_RX_TUNE=1 python bench.py --only c1500 --steps 20 --no-cpu --no-check
step nt_c64 300 env PPTK_RX_TUNE=1 python bench.py --only c64 --steps 20 --no-cpu --no-check
step prof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python bench.py --only c1500 --steps 10 --no-cpu --no-check
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d gpurun_out/prof_fetch -o run --output-format csv -- python bench.py --only c1500 --steps 3 --warmup 1 --no-cpu --no-check
step prof_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d gpurun_out/prof_write -o run --output-format csv -- python bench.py --only c1500 --steps 3 --warmup 1 --no-cpu --no-check
cat gpurun_out/steps.log
