#!/bin/bash
# Round 4 final tree: the forced one-rank RCCL bench line (N > 1 code path on
# one GPU: process group, RCCL all-gather, gathered check, validate_line).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04dist
export TMPDIR=/tmp
PPTK_BENCH_FORCE_DIST=1 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04dist/bench_dist1.json 2> gpurun_out/r04dist/bench_dist1.log
rc=$?; echo "dist1 rc=$rc"; python3 -c "
import json, sys
sys.path.insert(0, '.')
import bench
d=json.loads([x for x in open('gpurun_out/r04dist/bench_dist1.json') if x.startswith('{')][-1])
print(d['value'], d['allgather'].get('rccl_ranks'), d['allgather'].get('gathered_check'), bench.validate_line(d))"
exit $rc
