#!/bin/bash
# (abl/libpptkrx_exp.so: make abvariant NAME=exp DEFS="-DPPTK_RX_EXPERIMENTS -DPPTK_RX_DIAG"; cp build/ab_exp/libpptkrx.so abl/libpptkrx_exp.so -- build/ is not sent to the GPU box)
# Round 3: where the C64 lane kernel's time goes (exp = diagnostics build:
# bit 16 no per-frame phase, bit 8 no record stores; output invalid).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS=exp=abl/libpptkrx_exp.so
timeout -k 10 200 python -u tools/ab.py c64 12:-1 exp:12:-1 exp:12:16 exp:12:8 exp:12:24 12:-1:c > gpurun_out/c64_ab.json 2> gpurun_out/c64_ab.log
rc=$?; echo "c64 rc=$rc"; cat gpurun_out/c64_ab.json
exit $rc
