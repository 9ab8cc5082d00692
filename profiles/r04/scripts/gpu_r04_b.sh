#!/bin/bash
# Round 4: fused rate limiter (tests, A/B time, PMC traffic) and the
# communicator containment tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py > gpurun_out/r04b/permit_tests.log 2>&1
rc=$?; echo "permit tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04b/permit_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/permit_run.py records,keys,keys_denying --ab > gpurun_out/r04b/permit_ab.json 2> gpurun_out/r04b/permit_ab.log
rc=$?; echo "permit ab rc=$rc"; cat gpurun_out/r04b/permit_ab.json | cut -c1-600
[ $rc -eq 0 ] || exit $rc
for run in keys keys_denying records; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r04b/pmc_${run}_$c -o run -- python3 tools/permit_run.py $run > gpurun_out/r04b/pmc_${run}_$c.log 2>&1
    rc=$?; echo "pmc $run $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm.py tests/test_examples.py -m gpu > gpurun_out/r04b/comm_tests.log 2>&1
rc=$?; echo "comm tests rc=$rc"; grep -E "passed|failed|Error|FAIL" gpurun_out/r04b/comm_tests.log | tail -8
exit $rc
