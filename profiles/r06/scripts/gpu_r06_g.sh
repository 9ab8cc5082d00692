#!/bin/bash
# Round 6: e2e with the process on the GPU's NUMA node vs unpinned.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
step numa 900 python -u tools/numa_probe.py || exit $?
