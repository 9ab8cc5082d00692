#!/bin/bash
# Round 5: the write-phase period of offset-described batches, in process:
# 0.75 (f075.so) vs 1.0 (this tree) of the estimated tile, against no phases
# (prev.so); CMIX on T16S6 and T16S7L, placed buffers, two passes.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
for k in 1 2; do
  AB_PLACE=1 AB_ROUNDS=6 AB_LIBS=prev=tools/ab_libs/prev.so,f075=tools/ab_libs/f075.so step ab_cmix_$k 300 python -u tools/ab.py cmix prev:3:-1 f075:3:-1 3:-1 prev:6:-1 f075:6:-1 6:-1 || exit $?
  grep '^{' $O/ab_cmix_$k.log > $O/ab_cmix_$k.json
  python3 -c "
import json; d=json.load(open('$O/ab_cmix_$k.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
done
