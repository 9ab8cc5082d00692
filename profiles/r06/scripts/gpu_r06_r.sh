#!/bin/bash
# Round 6: the oversubscribed grid as built (tiles per wave: lane kernel 4,
# offset-described streaming 8; write-phase period from the resident waves)
# against the previous product (persistent grids) and against other tiles
# per wave / a long write-phase period (experiment build knobs).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7
export AB_LIBS=old=tools/ab_r06/libpptkrx_r06coal.so,exp=tools/ab_r06/libpptkrx_exp.so
step cmix_prod 300 python -u tools/ab.py cmix 3:-1 old:3:-1 3:-1:c old:3:-1:c || exit $?
step c64_prod 300 python -u tools/ab.py c64 12:-1 old:12:-1 12:-1:c old:12:-1:c || exit $?
for t in 2 4 16; do
  PPTK_RX_GATHER_TPW=$t step cmix_tpw$t 300 python -u tools/ab.py cmix 3:-1 exp:3:-1 || exit $?
done
PPTK_RX_PHASE_TICKS=1000000 step cmix_longphase 300 python -u tools/ab.py cmix 3:-1 exp:3:-1 || exit $?
for t in 2 8; do
  PPTK_RX_LANE_TPW=$t step c64_tpw$t 300 python -u tools/ab.py c64 12:-1 exp:12:-1 12:-1:c exp:12:-1:c || exit $?
done
