#!/bin/bash
# Pipelined host batches (pptk_rx_batch_submit / _complete): the host-path
# GPU tests, then small LDP-sized batches synchronous vs two deep.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gt_host 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "host or ring or registered or pipelined or rx_loop"
for cfg in c64 c1500; do
  for t in 1 8; do
    step pipe_${cfg}_reg${t} 200 env E2E_SIZES=32,256,1024,4096,16384 E2E_OUT=reg E2E_GATHER_THREADS=$t python tools/e2e_small.py $cfg
  done
done
cat gpurun_out/steps.log
