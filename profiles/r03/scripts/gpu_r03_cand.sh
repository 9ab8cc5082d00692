#!/bin/bash
# Round 3: which interchangeable 1536-byte shapes win on the mixed configs
# (T16S6, T32S3, T32S3D7, T16S7L, T16S6D1, M6), placed buffers, in-process A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_PLACE=1
for cfg in cmix imix; do
  timeout -k 10 300 python -u tools/ab.py $cfg 3:-1 4:-1 8:-1 6:-1 9:-1 13:-1 > gpurun_out/cand_ab_$cfg.json 2> gpurun_out/cand_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/cand_ab_$cfg.json')); print({k:v['ms'] for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
  [ $rc -eq 0 ] || exit $rc
done
