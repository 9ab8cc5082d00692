#!/bin/bash
# In-process A/B of kernel settings on the GPU box, e.g.
#   gpurun -- bash scripts/gpu_ab.sh c1500 3:33 3:32 3:33:c
# (tools/ab.py; AB_LIBS / AB_BIN / AB_MIXED pass through the environment)
source scripts/gpu_steps.sh
export TMPDIR=/tmp
cfg=$1
shift
step ab_$cfg 400 python tools/ab.py $cfg "$@"
cat gpurun_out/steps.log
