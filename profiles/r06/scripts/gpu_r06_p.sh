#!/bin/bash
# Round 6: more blocks than are resident (experiment build,
# PPTK_RX_GRID_MULT): C64 around the best multiple, and the streaming
# configs (C1500, CMIX), each beside the product in one process.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
export AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so AB_PLACE=1 AB_ROUNDS=7
for g in 8 32; do
  PPTK_RX_GRID_MULT=$g step c64_gm$g 300 python -u tools/ab.py c64 12:-1 exp:12:-1 12:-1:c exp:12:-1:c || exit $?
done
for g in 2 4 16; do
  PPTK_RX_GRID_MULT=$g step c1500_gm$g 300 python -u tools/ab.py c1500 -1:-1 exp:-1:-1 || exit $?
  PPTK_RX_GRID_MULT=$g step cmix_gm$g 300 python -u tools/ab.py cmix 3:-1 exp:3:-1 || exit $?
done
