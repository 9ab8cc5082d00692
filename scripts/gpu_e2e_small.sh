#!/bin/bash
# Host path: small LDP-sized calls (per-call latency) and 1 M-frame calls,
# current library against the previous build, record array registered.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gt_host 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "host or ring or registered"
for cfg in c1500 c64; do
  for t in 1 8; do
    step s_${cfg}_reg${t} 200 env E2E_SIZES=32,256,1024,4096,16384 E2E_OUT=reg E2E_GATHER_THREADS=$t python tools/e2e_small.py $cfg
    step s_${cfg}_reg${t}old 200 env E2E_SIZES=32,256,1024,4096,16384 E2E_OUT=reg E2E_GATHER_THREADS=$t E2E_LIB=abl/old/libpptkrx.so python tools/e2e_small.py $cfg
  done
done
for r in 1 2; do
  step e2e_new_$r 200 env E2E_REG_OUT=1 python tools/e2e.py
  step e2e_old_$r 200 env E2E_REG_OUT=1 E2E_LIB=abl/old/libpptkrx.so python tools/e2e.py
done
cat gpurun_out/steps.log
