#!/bin/bash
# Round 6: C64 (coalesced lane kernel) with more blocks than are resident
# (experiment build, PPTK_RX_GRID_MULT), each beside the product.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
export AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so AB_PLACE=1 AB_ROUNDS=7
for g in 2 4 16 64; do
  PPTK_RX_GRID_MULT=$g step gm$g 300 python -u tools/ab.py c64 12:-1 exp:12:-1 12:-1:c exp:12:-1:c || exit $?
done
