#!/bin/bash
# Round 3: M6 variant A/B (AB_LIBS old = the committed M6), then its parity tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS=old=abl/libpptkrx_old.so
for cfg in imix cmix; do
  timeout -k 10 200 python -u tools/ab.py $cfg 3:-1 13:-1 old:13:-1 > gpurun_out/m6b_ab_$cfg.json 2> gpurun_out/m6b_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/m6b_ab_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "forced_variant or compact_records or mixed_shape or fresh" > gpurun_out/m6b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/m6b_tests.log
exit $rc
