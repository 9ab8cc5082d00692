#!/bin/bash
# Round 4: fused rate limiter v2 (tests, A/B, phase stamps, traffic), comm tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py > gpurun_out/r04c/permit_tests.log 2>&1
rc=$?; echo "permit tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04c/permit_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/permit_run.py --stamps > gpurun_out/r04c/stamps.json 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/r04c/stamps.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/permit_run.py keys,keys_denying --ab > gpurun_out/r04c/permit_ab.json 2> gpurun_out/r04c/permit_ab.log
rc=$?; echo "permit ab rc=$rc"
[ $rc -eq 0 ] || exit $rc
for run in keys keys_denying; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r04c/pmc_${run}_$c -o run -- python3 tools/permit_run.py $run > gpurun_out/r04c/pmc_${run}_$c.log 2>&1
    rc=$?; echo "pmc $run $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm.py tests/test_examples.py -m gpu > gpurun_out/r04c/comm_tests.log 2>&1
rc=$?; echo "comm tests rc=$rc"; grep -E "passed|failed|Error|FAIL" gpurun_out/r04c/comm_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab.py cmix 3:0 14:0 3:0 14:0 13:0 > gpurun_out/r04c/ab_cmix.json 2> gpurun_out/r04c/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"; cat gpurun_out/r04c/ab_cmix.json | cut -c1-700
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab.py c1500 4:1 14:1 3:1 > gpurun_out/r04c/ab_c1500.json 2> gpurun_out/r04c/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"; cat gpurun_out/r04c/ab_c1500.json | cut -c1-700
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/scripts/gpu_r04_sq.sh
