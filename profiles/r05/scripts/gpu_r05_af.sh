#!/bin/bash
# Round 5: the record copy-back by DMA on the slot's second stream as the
# product path for large staged chunks into a registered record array: GPU
# suite, then host-to-host C64 (4 M frames, registered) and the LDP-sized
# batches against the previous tree (head.so); separate processes,
# alternating, two passes.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05af
mkdir -p $O
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
for r in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then export E2E_LIB=tools/ab_libs/head.so; else unset E2E_LIB; fi
    E2E_CFGS=c64 E2E_REG_OUT=1 step e2e_c64_${v}_$r 200 python -u tools/e2e.py 4194304 65536 || exit $?
    grep '^{' $O/e2e_c64_${v}_$r.log | tail -1
    E2E_DEPTH=4 E2E_SIZES=256,1024,4096 step small_${v}_$r 200 python -u tools/e2e_small.py c64 || exit $?
    grep '^{' $O/small_${v}_$r.log | tail -1 | cut -c1-400
  done
done
