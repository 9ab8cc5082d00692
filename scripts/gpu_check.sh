#!/bin/bash
# Quick whole-tree check on one box: GPU suite, smoke, default bench.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py
cat gpurun_out/steps.log
