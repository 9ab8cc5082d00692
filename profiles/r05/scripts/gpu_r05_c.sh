#!/bin/bash
# Round 5, third box: the rate limiter's launch order as the launch's own
# stop event (A/B: none / event record / stop event / round 4), the changed
# GPU tests, the forced one-rank RCCL bench line with the gather probe after
# the ring scrub.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_permit.py tests/test_gpu_comm.py tests/test_examples.py -m gpu > gpurun_out/r05c/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r05c/gputests.log | tail -2
[ $rc -eq 0 ] || exit $rc
for tok in 1048576 128; do
AB_KEYS=1 AB_TOKENS=$tok AB_ROUNDS=8 AB_LIBS=order0=tools/ab_libs/order0.so,r04=tools/ab_libs/r04.so timeout -k 10 300 python -u tools/ab_permit.py > gpurun_out/r05c/ab_permit_$tok.json 2> gpurun_out/r05c/ab_permit_$tok.log
rc=$?; echo "ab_permit $tok rc=$rc"; cat gpurun_out/r05c/ab_permit_$tok.json
[ $rc -eq 0 ] || exit $rc
done
PPTK_BENCH_FORCE_DIST=1 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu --no-live-pmc --detail gpurun_out/r05c/dist1_detail.json > gpurun_out/r05c/bench_dist1.json 2> gpurun_out/r05c/bench_dist1.log
rc=$?; echo "dist1 rc=$rc"; tail -c 1200 gpurun_out/r05c/bench_dist1.json
[ $rc -eq 0 ] || exit $rc
for cfg in cmix c1500; do
AB_PLACE=1 AB_ROUNDS=6 AB_LIBS=wgf=tools/ab_libs/wgflush.so timeout -k 10 300 python -u tools/ab.py $cfg 3:-1 wgf:3:-1 > gpurun_out/r05c/ab_wgflush_$cfg.json 2> gpurun_out/r05c/ab_wgflush_$cfg.log
rc=$?; echo "ab wgflush $cfg rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/r05c/ab_wgflush_$cfg.json')); print({k: v for k, v in d.items() if ':' in k})"
[ $rc -eq 0 ] || exit $rc
done
exit $rc
