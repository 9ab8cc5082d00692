#!/bin/bash
# Round 6: waves per block (PPTK_RX_WPB builds 1 and 2 against the
# product's 4): smaller blocks let the dispatcher refill a CU as soon as
# one wave's tiles are done.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7 AB_LIBS=w1=tools/ab_r06/libpptkrx_wpb1.so,w2=tools/ab_r06/libpptkrx_wpb2.so
step cmix 400 python -u tools/ab.py cmix 3:-1 w1:3:-1 w2:3:-1 6:-1 w1:6:-1 w2:6:-1 13:-1 w1:13:-1 w2:13:-1 || exit $?
step c64 300 python -u tools/ab.py c64 12:-1 w1:12:-1 w2:12:-1 12:-1:c w1:12:-1:c w2:12:-1:c || exit $?
step c1500 400 python -u tools/ab.py c1500 4:-1 w1:4:-1 w2:4:-1 6:-1 w1:6:-1 w2:6:-1 || exit $?
step imix 300 python -u tools/ab.py imix 13:-1 w1:13:-1 w2:13:-1 || exit $?
