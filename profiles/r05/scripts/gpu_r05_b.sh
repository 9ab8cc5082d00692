#!/bin/bash
# Round 5, second box: GPU suite (placed gather buffers, two queues' rings,
# rx_multigpu on library rings), the rate limiter's launch-order cost (A/B
# against the round-4 library and a build without the order), the forced
# one-rank RCCL bench line, then the default bench line (compact, e2e).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/r05b/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r05b/gputests.log | tail -2
[ $rc -eq 0 ] || exit $rc
for tok in 1048576 128; do
AB_KEYS=1 AB_TOKENS=$tok AB_ROUNDS=6 AB_LIBS=noorder=tools/ab_libs/noorder.so,r04=tools/ab_libs/r04.so timeout -k 10 300 python -u tools/ab_permit.py > gpurun_out/r05b/ab_permit_$tok.json 2> gpurun_out/r05b/ab_permit_$tok.log
rc=$?; echo "ab_permit $tok rc=$rc"; cat gpurun_out/r05b/ab_permit_$tok.json
[ $rc -eq 0 ] || exit $rc
done
PPTK_BENCH_FORCE_DIST=1 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu --no-live-pmc --detail gpurun_out/r05b/dist1_detail.json > gpurun_out/r05b/bench_dist1.json 2> gpurun_out/r05b/bench_dist1.log
rc=$?; echo "dist1 rc=$rc"; tail -c 1500 gpurun_out/r05b/bench_dist1.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --detail gpurun_out/r05b/bench_detail.json > gpurun_out/r05b/bench.json 2> gpurun_out/r05b/bench.log
rc=$?; echo "bench rc=$rc"; tail -c 3500 gpurun_out/r05b/bench.json
exit $rc
