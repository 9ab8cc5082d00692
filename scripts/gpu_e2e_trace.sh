#!/bin/bash
# Host path timeline: kernel and copy trace of the C64 end-to-end runs.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
export E2E_CFGS=c64
step e2e_trace_staged 200 env E2E_MODES=staged rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2e_tr_staged -o run --output-format csv -- python tools/e2e.py
step e2e_trace_ring 200 env E2E_MODES=ring rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2e_tr_ring -o run --output-format csv -- python tools/e2e.py
cat gpurun_out/steps.log
