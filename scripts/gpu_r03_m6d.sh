#!/bin/bash
# Round 3: M6 ring depth / occupancy A/B: D=3 at 2 waves/SIMD (product)
# against D=2 at 3 and at 2 waves/SIMD.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS=d1w3=abl/libpptkrx_d1w3.so,d2w2=abl/libpptkrx_d2w2.so
for cfg in imix cmix; do
  timeout -k 10 200 python -u tools/ab.py $cfg 3:-1 13:-1 d1w3:13:-1 d2w2:13:-1 > gpurun_out/m6d_ab_$cfg.json 2> gpurun_out/m6d_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/m6d_ab_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
