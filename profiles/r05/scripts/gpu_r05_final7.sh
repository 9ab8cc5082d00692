#!/bin/bash
# Round 5, the tree as committed last: the default bench line (untraced; its
# own same-run PMC passes give roofline.traffic).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05final7
mkdir -p $O
step bench 900 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('mix_sol_frac'), {k: v.get('kernel_ms') for k, v in d['configs'].items()})"
