#!/bin/bash
# Round 5, the tree as committed last: the whole GPU suite and smoke (after
# the rate limiter's grid under the split and the bench's unsplit fallback),
# then the forced one-rank line with the split.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05final6
mkdir -p $O
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
export PPTK_BENCH_FORCE_DIST=1 PPTK_BENCH_COLL_CUS=32
step bench_dist1_split 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu --no-live-pmc --detail $O/dist1_split_detail.json || exit $?
grep '^{' $O/bench_dist1_split.log | tail -1 > $O/bench_dist1_split.json
python3 -c "
import json; d=json.load(open('$O/bench_dist1_split.json')); print(d['value'], d['value_no_gather'], d['allgather'])"
