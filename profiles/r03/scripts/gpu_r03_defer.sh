#!/bin/bash
# (the PPTK_RX_DEFER_FLUSH variant was measured and removed from the source: DESIGN.md section 10)
# Round 3: deferred record flush (abl/libpptkrx_defer.so = make abvariant
# NAME=defer DEFS=-DPPTK_RX_DEFER_FLUSH) against the product library,
# in-process interleaved A/B on placed buffers.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS=defer=abl/libpptkrx_defer.so AB_PLACE=1
for cfg in cmix c1500 jmix; do
  timeout -k 10 300 python -u tools/ab.py $cfg -1:-1 defer:-1:-1 3:-1 defer:3:-1 > gpurun_out/defer_ab_$cfg.json 2> gpurun_out/defer_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/defer_ab_$cfg.json')); print({k:v for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
  [ $rc -eq 0 ] || exit $rc
done
