#!/bin/bash
# Round 4: communicator containment (abort during create, pending abort,
# bounded warm-up gather) and the C examples.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm.py tests/test_examples.py -m gpu > gpurun_out/comm_tests.log 2>&1
rc=$?; echo "comm tests rc=$rc"; grep -E "passed|failed|Error|FAIL" gpurun_out/comm_tests.log | tail -8
exit $rc
