#!/bin/bash
# Round 6: a short tail region on the oversubscribed grids (experiment
# build: the last PPTK_RX_TAIL_PCT % of the tiles at PPTK_RX_TAIL_TPW tiles
# per wave, dispatched last) beside the product (one region); then the wave
# concurrency of the best setting (probe build).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7 AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so
for p in 5 10 20; do
  for t in 1 2; do
    PPTK_RX_TAIL_PCT=$p PPTK_RX_TAIL_TPW=$t step cmix_p${p}_t$t 300 python -u tools/ab.py cmix 3:-1 exp:3:-1 6:-1 exp:6:-1 || exit $?
  done
done
PPTK_RX_TAIL_PCT=10 PPTK_RX_TAIL_TPW=1 step c64_p10_t1 300 python -u tools/ab.py c64 12:-1 exp:12:-1 12:-1:c exp:12:-1:c || exit $?
PPTK_RX_LIB=tools/ab_r06/libpptkrx_wt.so PPTK_RX_TAIL_PCT=10 PPTK_RX_TAIL_TPW=1 step wt_tail 300 python -u tools/wave_times.py cmix || exit $?
