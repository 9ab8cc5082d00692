#!/bin/bash
# Round 6: the speed-of-light search with oversubscribed grids (32 and 128
# blocks per CU) beside the product, every shape's time (RWMIX_SOL_SHAPES).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ad
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=5 AB_SOL=1 RWMIX_SOL_SHAPES=1
for c in cmix c64 c1500; do
  step sol_$c 400 python -u tools/ab.py $c -1:-1 || exit $?
done
