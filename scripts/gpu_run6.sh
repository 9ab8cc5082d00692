#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu
# variants: 3=T16S6 4=T32S3 5=T64S2 6=T16S7L 7=T32S4L ; flags bit0 NT
step ab_c1500 600 python tools/ab.py c1500 3:0 3:1 4:0 4:1 5:0 5:1 6:0 6:1 7:0 7:1
step ab_c1500a 600 python tools/ab.py c1500a 3:0 3:1 6:0 6:1 7:0 7:1
step ab_c64 600 python tools/ab.py c64 0:0 0:1 0:2 1:0 2:0
cat gpurun_out/ab_*.log | grep '^{'
