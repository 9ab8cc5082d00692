#!/bin/bash
# Round 6 closing tree (the final tree: tile ranges, SOL search with oversubscribed grids): the whole GPU suite, smoke, the default bench line
# (untraced; its own same-run PMC passes give roofline.traffic), then the
# N > 1 code path on one GPU (a one-rank RCCL communicator) split
# (PPTK_BENCH_COLL_CUS=32, as N > 1 runs: the split made before the
# communicator, whose blocks the library caps at 32; no NCCL_* variable).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06close3
mkdir -p $O
step gputests 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu || exit $?
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 900 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
export PPTK_BENCH_FORCE_DIST=1
PPTK_BENCH_COLL_CUS=32 step bench_dist1_split 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu --no-live-pmc --detail $O/dist1_split_detail.json || exit $?
grep '^{' $O/bench_dist1_split.log | tail -1 > $O/bench_dist1_split.json
