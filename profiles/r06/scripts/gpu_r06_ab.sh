#!/bin/bash
# Round 6: fixed-stride C1500 tiles per wave 16 / 32 / 64 (experiment build,
# PPTK_RX_FIXED_TPW) beside the product (persistent), T16S7L and T32S3.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ab
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=9 AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so
for t in 16 32 64; do
  PPTK_RX_FIXED_TPW=$t step c1500_t$t 400 python -u tools/ab.py c1500 6:-1 exp:6:-1 4:-1 exp:4:-1 6:-1:c exp:6:-1:c || exit $?
done
