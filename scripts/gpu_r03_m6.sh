#!/bin/bash
# (abl/libpptkrx_exp.so: make abvariant NAME=exp DEFS="-DPPTK_RX_EXPERIMENTS -DPPTK_RX_DIAG"; cp build/ab_exp/libpptkrx.so abl/libpptkrx_exp.so -- build/ is not sent to the GPU box)
# Round 3: the mixed-shape kernel (RX_M6): parity tests, then in-process A/B
# against the automatic team shape on the mixed configs (exp = diagnostics
# build: bit 16 no lane phase, bit 8 no record stores; output invalid).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "forced_variant or compact_records or mixed_shape or fresh or autotune or mixed_length or frag" > gpurun_out/m6_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/m6_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
export AB_LIBS=exp=abl/libpptkrx_exp.so
for cfg in imix cmix; do
  timeout -k 10 200 python -u tools/ab.py $cfg 3:-1 13:-1 exp:3:24 exp:13:24 exp:13:16 exp:13:8 > gpurun_out/m6_ab_$cfg.json 2> gpurun_out/m6_ab_$cfg.log
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/m6_ab_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
