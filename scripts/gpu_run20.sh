#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 6
step chk_c1500b 300 python tools/check_rec32.py c1500
cat gpurun_out/steps.log
