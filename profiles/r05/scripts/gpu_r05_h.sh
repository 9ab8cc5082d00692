#!/bin/bash
# Round 5: LDP-sized host batches on this round's tree (tools/e2e_small.py,
# synchronous and pipelined four deep), C64.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05h
export TMPDIR=/tmp
E2E_DEPTH=4 timeout -k 10 300 python -u tools/e2e_small.py c64 > gpurun_out/r05h/e2e_small_c64.json 2> gpurun_out/r05h/e2e_small_c64.log
rc=$?; echo "e2e_small rc=$rc"; head -c 2500 gpurun_out/r05h/e2e_small_c64.json
exit $rc
