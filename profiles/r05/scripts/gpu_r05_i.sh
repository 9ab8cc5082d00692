#!/bin/bash
# Round 5: LDP-sized host batches, this tree against the round-2/3/4 libraries
# (process-level, two interleaved passes; tools/e2e_small.py, C64, four deep).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05i
export TMPDIR=/tmp
for pass in 1 2; do
for lib in cur r04 r03 r02; do
  if [ $lib = cur ]; then unset E2E_LIB; else export E2E_LIB=tools/ab_libs/$lib.so; fi
  E2E_DEPTH=4 E2E_SIZES=256,1024,4096 timeout -k 10 200 python -u tools/e2e_small.py c64 > gpurun_out/r05i/e2e_${lib}_$pass.json 2> gpurun_out/r05i/e2e_${lib}_$pass.log
  rc=$?; echo "$lib pass $pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json; d=json.load(open('gpurun_out/r05i/e2e_${lib}_$pass.json')); print({k: v for k, v in d.items() if k.startswith(('staged_', 'pipe_staged_'))})"
done
done
