#!/bin/bash
# Round 4: fused rate limiter v4 (speculative verdicts, early exit).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04g
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py > gpurun_out/r04g/permit_tests.log 2>&1
rc=$?; echo "permit tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04g/permit_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/permit_run.py --stamps > gpurun_out/r04g/stamps.json 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/r04g/stamps.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/permit_run.py keys,keys_denying --ab > gpurun_out/r04g/permit_ab.json 2> gpurun_out/r04g/permit_ab.log
rc=$?; echo "permit ab rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r04g/permit_ab.json'):
    d=json.loads(l)
    for k,v in d.items(): print(k, v['keys']['ms_per_batch'], v['keys_denying']['ms_per_batch'])"
[ $rc -eq 0 ] || exit $rc
for run in keys keys_denying; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r04g/pmc_${run}_$c -o run -- python3 tools/permit_run.py $run > gpurun_out/r04g/pmc_${run}_$c.log 2>&1
    rc=$?; echo "pmc $run $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
PPTK_BENCH_FORCE_DIST=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04g/bench_dist1.json 2> gpurun_out/r04g/bench_dist1.log
rc=$?; echo "dist1 rc=$rc"; tail -c 1500 gpurun_out/r04g/bench_dist1.json
[ $rc -eq 0 ] || exit $rc
