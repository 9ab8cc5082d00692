#!/bin/bash
# Round 6: C64 on the coalesced lane kernel with fewer resident blocks per
# CU (experiment build, PPTK_RX_BPC), each beside the product in one process.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
export AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so AB_PLACE=1 AB_ROUNDS=7
for b in 1 2 3; do
  PPTK_RX_BPC=$b step bpc$b 300 python -u tools/ab.py c64 12:-1 exp:12:-1 12:-1:c exp:12:-1:c || exit $?
done
PPTK_RX_GRID_MULT=2 step gm2 300 python -u tools/ab.py c64 12:-1 exp:12:-1 || exit $?
