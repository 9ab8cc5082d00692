#!/bin/bash
# The default bench command, twice, on one box (profiles/r02/boxes).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step bench_a 600 python bench.py
step bench_b 600 python bench.py
cat gpurun_out/steps.log
