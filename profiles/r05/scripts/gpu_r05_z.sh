#!/bin/bash
# Round 5: write phases, offset batches with the whole estimated tile as
# period: GPU suite, smoke, the default bench line, the forced one-rank line,
# then A/B against the library without phases (prev.so), CMIX and C1500.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 900 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']); print({k: (v.get('kernel_ms'), v.get('frac'), v.get('sol_frac'), v.get('variant')) for k, v in d['configs'].items()})"
export PPTK_BENCH_FORCE_DIST=1
step bench_dist1 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu --no-live-pmc --detail $O/dist1_detail.json || exit $?
unset PPTK_BENCH_FORCE_DIST
grep '^{' $O/bench_dist1.log | tail -1 > $O/bench_dist1.json
python3 -c "
import json; d=json.load(open('$O/bench_dist1.json')); print(d['value'], d['value_no_gather'], d['allgather']['overlap_loss'])"
for cfg in cmix c1500; do
  AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=prev=tools/ab_libs/prev.so step ab_$cfg 300 python -u tools/ab.py $cfg prev:-1:-1 -1:-1 prev:6:-1 6:-1 || exit $?
  grep '^{' $O/ab_$cfg.log > $O/ab_$cfg.json
  python3 -c "
import json; d=json.load(open('$O/ab_$cfg.json')); print('$cfg', {k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
done
