#!/bin/bash
# Fused length-group launch diagnostics: one group only (c1500g, all frames
# in the 1521-byte group).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
export AB_LIBS=old=abl/old/libpptkrx.so
step ab_c1500g 300 env AB_PLACE=1 python tools/ab.py c1500g -1:-1 -1:-1:m old:-1:-1:m old:-1:-1
cat gpurun_out/steps.log
