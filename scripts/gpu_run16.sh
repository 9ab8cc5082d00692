#!/bin/bash
# CMIX identity-order variant/flag sweep; C64 variant/flag sweep.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step ab_cmix_sweep 400 python tools/ab.py cmix 3:0 3:1 3:32 3:33 4:0 4:1 5:0 5:1 6:0 9:0 8:0 2:0
step ab_c64_sweep 300 python tools/ab.py c64 0:0 0:1 0:32 0:33 0:2 1:0 10:0
cat gpurun_out/steps.log
