#!/bin/bash
# Round 6: oversubscribed grids (experiment build, PPTK_RX_GRID_MULT) on the
# streaming shapes, forced: CMIX T16S6 over more multiples, C1500 T32S3 and
# T16S6; each beside the product in one process.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
export AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so AB_PLACE=1 AB_ROUNDS=7
for g in 8 32 64; do
  PPTK_RX_GRID_MULT=$g step cmix_gm$g 300 python -u tools/ab.py cmix 3:-1 exp:3:-1 3:-1:c exp:3:-1:c || exit $?
done
for g in 4 16; do
  PPTK_RX_GRID_MULT=$g step c1500_gm$g 300 python -u tools/ab.py c1500 4:-1 exp:4:-1 3:-1 exp:3:-1 || exit $?
done
