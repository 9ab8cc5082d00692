#!/bin/bash
# Round 6: fixed-stride C1500 on oversubscribed grids for the line-aligned
# shapes (experiment build, PPTK_RX_FIXED_TPW), beside the product
# (persistent); then the whole -m gpu suite on the product after the tile
# range rework.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7 AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so
for t in 8 32; do
  PPTK_RX_FIXED_TPW=$t step c1500_t$t 400 python -u tools/ab.py c1500 6:-1 exp:6:-1 7:-1 exp:7:-1 4:-1 exp:4:-1 || exit $?
done
step suite 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ || exit $?
