#!/bin/bash
# Round 6: the last tile of each wave waits for its write phase too
# (PPTK_RX_END_WAIT build) against the product, CMIX shapes and C1500.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ak
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=9 AB_LIBS=ew=tools/ab_r06/libpptkrx_endwait.so
step cmix 400 python -u tools/ab.py cmix 3:-1 ew:3:-1 6:-1 ew:6:-1 || exit $?
step c1500 400 python -u tools/ab.py c1500 6:-1 ew:6:-1 4:-1 ew:4:-1 || exit $?
