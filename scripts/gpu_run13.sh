#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu
step e2e8 600 env E2E_GATHER_THREADS=8 python tools/e2e.py 1048576 65536
step e2e16 600 env E2E_GATHER_THREADS=16 python tools/e2e.py 1048576 65536
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
cat gpurun_out/steps.log
