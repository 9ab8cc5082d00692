#!/bin/bash
# Rate limiter: GPU tests, in-process A/B against the previous library, and
# a kernel trace of the new one.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
export AB_LIBS=old=abl/old/libpptkrx.so
step gt_permit 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "permit"
step ab_permit 300 python tools/ab_permit.py
step tr_permit 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_permit -o run --output-format csv -- python tools/ab_permit.py
cat gpurun_out/steps.log
