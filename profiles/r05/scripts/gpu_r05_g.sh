#!/bin/bash
# Round 5: the HBM side of C8G emulated on one GPU (tools/c8g_emul.py), and
# the N-rank gather probe test.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05g
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_comm.py -k "gather_alloc" -m gpu > gpurun_out/r05g/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05g/tests.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/c8g_emul.py 20 > gpurun_out/r05g/c8g_emul.json 2> gpurun_out/r05g/c8g_emul.log
rc=$?; echo "c8g_emul rc=$rc"; head -c 2500 gpurun_out/r05g/c8g_emul.json
exit $rc
