#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step ab_w 600 python tools/ab.py c1500 3:0 3:32 3:64 3:1 3:33 3:65 3:8 3:9
step ab_w64 600 python tools/ab.py c64 0:0 0:32 0:64 0:8
cat gpurun_out/ab_*.log | grep '^{'
