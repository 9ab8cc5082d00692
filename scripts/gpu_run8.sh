#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step ab_st 600 python tools/ab.py c1500 3:0 3:1 3:32 3:33 3:128 3:129 3:9 6:33 6:1
step ab_st64 600 python tools/ab.py c64 0:0 0:32 0:128 0:8 0:24
cat gpurun_out/ab_*.log | grep '^{'
