#!/bin/bash
# Round 6: uniform host chunks as fixed-stride batches (no descriptors), the
# ring check on the worker pool: the host-path tests, then bench's e2e.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step host 600 $PT -m gpu tests/test_gpu_parity.py -k "host_batch or ring" tests/test_examples.py || exit $?
step e2e 600 python -u -c "
import json, torch, bench
print(json.dumps(bench.e2e_bench(torch.device('cuda:0'))))" || exit $?
