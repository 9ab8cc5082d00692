#!/bin/bash
# Round 5: the rate limiter's one-launch path on the split batches' stream
# (its grid barriers need every workgroup resident: the grid now leaves out
# the collective's CUs), test_stream_split; and the permit suite.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05au
mkdir -p $O
step tests 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k stream_split tests/test_gpu_permit.py || exit $?
tail -2 $O/tests.log
