#!/bin/bash
# Round 6: the C64 lane kernel with more waves per SIMD (builds without the
# next-tile prefetch at 4 / 5 / 6 waves, and with it at 5; all spill a
# little) against the product (prefetch, 4 waves), placed buffers.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ah
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7 AB_LIBS=p0w4=tools/ab_r06/libpptkrx_p0w4.so,p0w5=tools/ab_r06/libpptkrx_p0w5.so,p0w6=tools/ab_r06/libpptkrx_p0w6.so,p1w5=tools/ab_r06/libpptkrx_p1w5.so
step c64 400 python -u tools/ab.py c64 12:-1 p0w4:12:-1 p0w5:12:-1 p0w6:12:-1 p1w5:12:-1 12:-1:c p0w4:12:-1:c p0w5:12:-1:c p0w6:12:-1:c p1w5:12:-1:c || exit $?
