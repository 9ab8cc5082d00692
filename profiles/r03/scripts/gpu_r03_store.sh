#!/bin/bash
# Round 3: CMIX record-store policy A/B on the current kernels (flags: 32 NT
# stores = default, 0 plain, 64 sc1 write-through, 2 no LDS staging), placed
# buffers, then the same on C1500.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_PLACE=1
for cfg in cmix c1500; do
  timeout -k 10 300 python -u tools/ab.py $cfg 3:32 3:0 3:64 3:34 4:33 4:1 > gpurun_out/store_ab_$cfg.json 2> gpurun_out/store_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/store_ab_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
