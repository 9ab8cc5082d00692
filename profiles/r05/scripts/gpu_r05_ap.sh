#!/bin/bash
# Round 5: when does each wave of the persistent rx grid finish?  Probe
# build with per-wave start/end clocks (tools/wave_times.py, ab_libs/wt.so).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ap
mkdir -p $O
PPTK_RX_LIB=tools/ab_libs/wt.so step wave_times 400 python -u tools/wave_times.py || exit $?
grep -h '^{' $O/wave_times.log
