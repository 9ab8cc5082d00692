#!/bin/bash
# Round 5: the new dense-hash parity test, then the whole GPU suite.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05j
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "dense_hash" -m gpu > gpurun_out/r05j/hash_tests.log 2>&1
rc=$?; echo "hash tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05j/hash_tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r05j/hash_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/r05j/gputests.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" gpurun_out/r05j/gputests.log | tail -1
exit $rc
