#!/bin/bash
# Round 3: M6 at D = 1, 3 waves/SIMD (product): parity tests, A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/m6c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/m6c_tests.log
[ $rc -eq 0 ] || exit $rc
for cfg in imix cmix jmix; do
  timeout -k 10 200 python -u tools/ab.py $cfg 3:-1 13:-1 9:-1 > gpurun_out/m6c_ab_$cfg.json 2> gpurun_out/m6c_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/m6c_ab_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
