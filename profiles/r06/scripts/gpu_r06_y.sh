#!/bin/bash
# Round 6: every wave's start and end (probe build, PPTK_RX_WAVE_TIMES) on
# the oversubscribed grids and, for comparison, on persistent ones: how many
# waves run at once over the launch and how long its tail is.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
export PPTK_RX_LIB=tools/ab_r06/libpptkrx_wt.so
step wt_over 300 python -u tools/wave_times.py cmix c64 || exit $?
PPTK_RX_GATHER_TPW=0 PPTK_RX_LANE_TPW=0 step wt_persist 300 python -u tools/wave_times.py cmix c64 || exit $?
