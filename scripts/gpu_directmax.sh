#!/bin/bash
# PPTK_RX_DIRECT_MAX_BYTES with four slots in flight: large calls (e2e.py)
# and LDP-sized calls (e2e_small.py, synchronous and four deep).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
for dm in 8388608 4194304 2097152 1048576; do
  step dmL_$dm 200 env E2E_REG_OUT=1 PPTK_RX_DIRECT_MAX_BYTES=$dm python tools/e2e.py
  for cfg in c64 c1500; do
    step dmS_${cfg}_$dm 200 env E2E_SIZES=1024,4096,16384 E2E_OUT=reg E2E_DEPTH=4 PPTK_RX_DIRECT_MAX_BYTES=$dm python tools/e2e_small.py $cfg
  done
done
cat gpurun_out/steps.log
