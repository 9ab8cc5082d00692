#!/bin/bash
# Round 5: host-to-host C64 (4 M frames, record array registered): gather
# threads 8 / 16 and chunks of 64 K / 256 K frames (tools/e2e.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05s
export TMPDIR=/tmp
for gt in 8 16; do
  for ch in 65536 262144; do
    E2E_CFGS=c64 E2E_REG_OUT=1 E2E_GATHER_THREADS=$gt timeout -k 10 200 python -u tools/e2e.py 4194304 $ch > gpurun_out/r05s/e2e_c64_t${gt}_c${ch}.json 2> gpurun_out/r05s/e2e_c64_t${gt}_c${ch}.log
    rc=$?; echo "e2e c64 threads $gt chunk $ch rc=$rc"; cat gpurun_out/r05s/e2e_c64_t${gt}_c${ch}.json
    [ $rc -eq 0 ] || exit $rc
  done
done
