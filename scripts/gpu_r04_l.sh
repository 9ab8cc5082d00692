#!/bin/bash
# Round 4: fused rate limiter phase-3 stamps (codes staged, boundaries found).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/permit_run.py --stamps > gpurun_out/r04l/stamps.json 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/r04l/stamps.json
[ $rc -eq 0 ] || exit $rc
