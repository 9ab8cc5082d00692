#!/bin/bash
# Round 6: CMIX on the oversubscribed grid -- tiles per wave and the
# write-phase period around the product's (8 tiles, ~13.4 us), for T16S6 and
# T16S7L (the shape the bench's autotune now picks); experiment build beside
# the product, one process per setting.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7 AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so
for t in 4 6 12; do
  PPTK_RX_GATHER_TPW=$t step tpw$t 300 python -u tools/ab.py cmix 3:-1 exp:3:-1 6:-1 exp:6:-1 || exit $?
done
for p in 1700 2100; do
  PPTK_RX_PHASE_TICKS=$p step ph$p 300 python -u tools/ab.py cmix 3:-1 exp:3:-1 6:-1 exp:6:-1 || exit $?
done
