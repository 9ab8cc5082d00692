#!/bin/bash
# (the own-lane round was measured and removed from the source: DESIGN.md section 10)
# Round 3: M6 with an own-lane round for frames of at most six chunks
# (abl/libpptkrx_old.so = the tree before it): parity, then in-process A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_frag.py -m gpu > gpurun_out/m6own_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/m6own_tests.log
[ $rc -eq 0 ] || exit $rc
export AB_LIBS=old=abl/libpptkrx_old.so
for cfg in imix cmix; do
  timeout -k 10 200 python -u tools/ab.py $cfg 3:-1 13:-1 old:13:-1 > gpurun_out/m6own_ab_$cfg.json 2> gpurun_out/m6own_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/m6own_ab_$cfg.json')); print({k:v for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
  [ $rc -eq 0 ] || exit $rc
done
