#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests -x -q -m gpu
cat gpurun_out/steps.log
