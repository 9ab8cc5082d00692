#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step chk_c1500 300 python tools/check_rec32.py c1500
step gputests 900 python -m pytest tests -x -q -m gpu
cat gpurun_out/steps.log
