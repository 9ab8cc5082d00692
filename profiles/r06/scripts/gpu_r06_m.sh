#!/bin/bash
# Round 6: coalesced lane-kernel tiles as the product: the lane-kernel and
# golden parity tests, then C64 in process against the per-frame-load build.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
step parity 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py || exit $?
export AB_LIBS=old=tools/ab_r06/libpptkrx_r06pre.so AB_PLACE=1 AB_ROUNDS=9 AB_SOL=1
step ab_c64 400 python -u tools/ab.py c64 12:-1 old:12:-1 12:-1:c old:12:-1:c || exit $?
