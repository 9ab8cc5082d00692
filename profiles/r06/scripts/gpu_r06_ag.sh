#!/bin/bash
# Round 6: the rate limiter beside oversubscribed receive batches.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ag
mkdir -p $O
step beside 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_permit.py -k "beside or two_contexts" || exit $?
