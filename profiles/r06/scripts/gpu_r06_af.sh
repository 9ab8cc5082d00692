#!/bin/bash
# Round 6: full-size windows against the oracle on the product's grids.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06af
mkdir -p $O
step windows 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "full_size" || exit $?
