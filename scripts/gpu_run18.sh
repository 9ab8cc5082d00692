#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step chk_c1500 300 python tools/check_rec32.py c1500
step chk_c64 300 python tools/check_rec32.py c64
step chk_cmix 300 python tools/check_rec32.py cmix
cat gpurun_out/steps.log
