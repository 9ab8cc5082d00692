#!/bin/bash
# Round 5: what the dense flow-hash writes cost beside the C1500 stream on
# the library's rings, and what decides it (tools/hash_probe.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/hash_probe.py 6 > gpurun_out/r05d/hash_probe.json 2> gpurun_out/r05d/hash_probe.log
rc=$?; echo "hash_probe rc=$rc"; cat gpurun_out/r05d/hash_probe.json | head -c 3000
exit $rc
