#!/bin/bash
# Round 5: global write phases -- C1500-shaped tiles on the library's placed
# rings with each record run written at its tile's end or held until a
# chip-wide clock period begins (tools/epoch_probe.py), beside the rx kernel;
# the XCDs writing in turn (EPOCH_SWEEP=stagger).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05u3
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/epoch_probe.py --out gpurun_out/r05u3/epoch.json > gpurun_out/r05u3/epoch.log 2>&1
rc=$?; echo "epoch rc=$rc"; cat gpurun_out/r05u3/epoch.json
exit $rc
