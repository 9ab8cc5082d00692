#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 5
for t in 0 1 2 3; do
  step c1500_t$t 300 env PPTK_RX_TUNE=$t python bench.py --only c1500 --steps 20 --no-cpu --no-check
  step c64_t$t 300 env PPTK_RX_TUNE=$t python bench.py --only c64 --steps 20 --no-cpu --no-check
done
step c1500_t32 300 env PPTK_RX_VARIANT=4 python bench.py --only c1500 --steps 20 --no-cpu --no-check
step c1500_t32_nt 300 env PPTK_RX_VARIANT=4 PPTK_RX_TUNE=1 python bench.py --only c1500 --steps 20 --no-cpu --no-check
step c64_t4s2 300 env PPTK_RX_VARIANT=1 python bench.py --only c64 --steps 20 --no-cpu --no-check
step c64_t16s2 300 env PPTK_RX_VARIANT=2 python bench.py --only c64 --steps 20 --no-cpu --no-check
grep -h "rank 0" gpurun_out/*.log
