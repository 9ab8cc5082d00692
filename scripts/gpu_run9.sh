#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step ab_d 600 python tools/ab.py c1500 3:0 3:8 4:0 4:8 8:0 8:8 9:0 9:8 8:1 8:9
cat gpurun_out/ab_*.log | grep '^{'
