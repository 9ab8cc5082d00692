#!/bin/bash
# Round 5: host-to-host C64 (4 M frames), records copied back (DMA) instead
# of written into a registered array, 8 gather threads, 64 K-frame chunks.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05s
export TMPDIR=/tmp
E2E_CFGS=c64 E2E_GATHER_THREADS=8 timeout -k 10 200 python -u tools/e2e.py 4194304 65536 > gpurun_out/r05s/e2e_c64_t8_c65536_copied.json 2> gpurun_out/r05s/e2e_c64_copied.log
rc=$?; echo "e2e c64 copied rc=$rc"; cat gpurun_out/r05s/e2e_c64_t8_c65536_copied.json
exit $rc
