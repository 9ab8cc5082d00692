#!/bin/bash
# Branch-free GATHER descriptors + length-group launches: parity, A/B against
# the previous build (build/ab_old), then a short bench.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
export AB_LIBS=old=build/ab_old/libpptkrx.so
step gputests 900 python -m pytest tests -x -q -m gpu
step ab_cmix 300 python tools/ab.py cmix 3:33 old:3:33 4:33 5:33 11:33
step ab_cmix_mixed 300 env AB_MIXED=1 AB_LIBS= python tools/ab.py cmix -1:-1 3:33 11:33 -1:0 -1:1
step ab_c1500g 300 python tools/ab.py c1500g 3:33 old:3:33
step bench 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 4
cat gpurun_out/steps.log
