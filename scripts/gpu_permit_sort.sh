#!/bin/bash
# Rate limiter sort shapes (PPTK_RX_PERMIT_SORT), each in its own process,
# interleaved, plus the permit GPU tests under every shape.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
for v in 2 4 5 6; do
  step gt_permit_$v 200 env PPTK_RX_PERMIT_SORT=$v python -u -m pytest tests/test_gpu_permit.py -x -q --timeout 120 --timeout-method thread
done
for r in 1 2; do
  for v in 2 4 5 6; do
    step ps_${v}_$r 200 env PPTK_RX_PERMIT_SORT=$v python tools/opbench.py permit --steps 10 --warmup 2
  done
done
cat gpurun_out/steps.log
