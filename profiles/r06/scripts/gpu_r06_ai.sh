#!/bin/bash
# Round 6: C64 host to host with the record array registered or not.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ai
mkdir -p $O
step e2e_regs 400 python -u tools/e2e_regs.py 2 || exit $?
