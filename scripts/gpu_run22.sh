#!/bin/bash
# Blocked tile order experiment.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "forced or compact"
step ab_c1500 300 python tools/ab.py c1500 3:33 3:289 3:32 3:288 3:33:c 3:289:c
step ab_c64 300 python tools/ab.py c64 0:32 0:288 0:32:c 0:288:c
step ab_cmix 300 python tools/ab.py cmix 3:32 3:288
cat gpurun_out/steps.log
