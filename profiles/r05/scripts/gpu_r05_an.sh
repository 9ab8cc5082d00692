#!/bin/bash
# Round 5: pptk_rx_stream_split (the batches and the all-gather on disjoint
# CUs) -- its GPU test, the comm tests, the RCCL stand-in beside C1500 with
# the product's split (32 / 64 CUs) and without, and the one-rank bench
# all-gather path with the split on.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05an
mkdir -p $O
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "stream_split or autotune_keeps" tests/test_gpu_comm.py || exit $?
step nosplit 300 python -u tools/c8g_emul.py 20 --standin 32 || exit $?
step split32 300 python -u tools/c8g_emul.py 20 --standin 16,32,64 --split 32 || exit $?
step split64 300 python -u tools/c8g_emul.py 20 --standin 32,64,128 --split 64 || exit $?
PPTK_BENCH_FORCE_DIST=1 step dist1 400 python -u bench.py --steps 20 --no-cpu --no-secondary --no-e2e --no-live-pmc --no-rec32 || exit $?
grep -h '^{' $O/nosplit.log $O/split32.log $O/split64.log
tail -1 $O/dist1.log | cut -c1-3000
