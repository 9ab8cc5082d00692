#!/bin/bash
# Round 3: DPP team sums in the team kernels (AB_LIBS old = LDS-shuffle team sums), then parity.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS=old=abl/libpptkrx_old.so
for cfg in cmix c1500 imix; do
  timeout -k 10 200 python -u tools/ab.py $cfg -1:-1 old:-1:-1 3:-1 old:3:-1 4:-1 old:4:-1 > gpurun_out/dpp_ab_$cfg.json 2> gpurun_out/dpp_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/dpp_ab_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/dpp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/dpp_tests.log
exit $rc
