#!/bin/bash
# (abl/libpptkrx_exp.so: make abvariant NAME=exp DEFS="-DPPTK_RX_EXPERIMENTS -DPPTK_RX_DIAG"; cp build/ab_exp/libpptkrx.so abl/libpptkrx_exp.so -- build/ is not sent to the GPU box)
# Round 3: where IMIX / CMIX time goes -- streaming shapes (same records) and
# diagnostic bits of the experiment build (16 = no lane phase, 8 = no record
# stores; output invalid), in-process interleaved A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS=exp=abl/libpptkrx_exp.so
for cfg in imix cmix; do
  timeout -k 10 300 python -u tools/ab.py $cfg 3:0 11:0 2:0 10:0 1:0 exp:3:0 exp:3:16 exp:3:8 exp:3:24 exp:2:24 exp:1:24 > gpurun_out/ab_$cfg.json 2> gpurun_out/ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/ab_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
