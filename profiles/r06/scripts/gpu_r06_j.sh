#!/bin/bash
# Round 6: staged chunks of equal-length frames at any host addresses run
# without descriptors -- the host-path parity tests and the C hosts.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
step host_tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "host or ring or uniform or compact" tests/test_examples.py || exit $?
