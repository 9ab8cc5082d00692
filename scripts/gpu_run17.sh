#!/bin/bash
# Compact records + layout-dependent memory policy: parity, bench, A/B.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests -x -q -m gpu
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 6
step ab_c1500 300 python tools/ab.py c1500 3:33 3:32 3:1 3:0
cat gpurun_out/steps.log
