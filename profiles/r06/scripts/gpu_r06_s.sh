#!/bin/bash
# Round 6: oversubscribed grids -- the whole -m gpu suite on the product,
# then M6 (CMIX, IMIX) and T64S2 (JMIX) with a few tiles per wave
# (experiment build, PPTK_RX_MIX_TPW) beside the product.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
step suite 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ || exit $?
export AB_PLACE=1 AB_ROUNDS=7 AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so
for t in 4 8; do
  PPTK_RX_MIX_TPW=$t step cmix_m6_tpw$t 300 python -u tools/ab.py cmix 13:-1 exp:13:-1 || exit $?
  PPTK_RX_MIX_TPW=$t step imix_m6_tpw$t 300 python -u tools/ab.py imix 13:-1 exp:13:-1 || exit $?
  PPTK_RX_MIX_TPW=$t step jmix_t64_tpw$t 300 python -u tools/ab.py jmix 5:-1 exp:5:-1 || exit $?
done
