#!/bin/bash
# Round 6: the tail chunk parked in LDS by the team (one store per round)
# against the in-round correction (every lane, every round) and the round-5
# kernel (second read of the chunk): full -m gpu suite first, then A/B.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step gpu 900 $PT -m gpu tests || exit $?
export AB_LIBS=r05=tools/ab_r06/libpptkrx_r05.so,reg=tools/ab_r06/libpptkrx_tailreg.so AB_PLACE=1 AB_ROUNDS=7
for cfg in cmix imix jmix c1500; do
  step ab_$cfg 300 python -u tools/ab.py $cfg -1:-1 reg:-1:-1 r05:-1:-1 || exit $?
done
# the shapes autotune picks between on mixed batches: T16S6 (3), M6 (13)
for cfg in cmix imix; do
  step ab_${cfg}_shapes 300 python -u tools/ab.py $cfg 3:-1 reg:3:-1 r05:3:-1 13:-1 reg:13:-1 r05:13:-1 || exit $?
done
