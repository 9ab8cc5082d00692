#!/bin/bash
# Pipelined host batches (pptk_rx_batch_submit / _complete): the host-path
# GPU tests, then small LDP-sized batches synchronous vs pipelined at
# depths 2, 3 and 4.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gt_host 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "host or ring or registered or pipelined or rx_loop or rx_mt"
for cfg in c64 c1500; do
  for d in 2 3 4; do
    step pipe_${cfg}_reg1_d${d} 200 env E2E_SIZES=32,256,1024,4096,16384 E2E_OUT=reg E2E_GATHER_THREADS=1 E2E_DEPTH=$d python tools/e2e_small.py $cfg
  done
done
cat gpurun_out/steps.log
