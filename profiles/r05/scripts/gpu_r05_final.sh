#!/bin/bash
# Round 5 closing tree, first box: the whole GPU suite, smoke, then the
# default bench line (untraced; its own same-run PMC passes give
# roofline.traffic), full result in $O/bench_detail.json.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 900 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
tail -c 600 $O/bench.json
# the N > 1 code path on one GPU: a one-rank RCCL communicator, the placed
# double-buffered gather buffers, the gathered check, bench.validate_line
export PPTK_BENCH_FORCE_DIST=1
step bench_dist1 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu --no-live-pmc --detail $O/dist1_detail.json || exit $?
unset PPTK_BENCH_FORCE_DIST
grep '^{' $O/bench_dist1.log | tail -1 > $O/bench_dist1.json
python3 -c "
import json; d=json.load(open('$O/bench_dist1.json')); print(d['value'], d['value_no_gather'], d['allgather']['overlap_loss'])"
