#!/bin/bash
# Round 5: SQ counters of the C64 launch (lane kernel L4, full and compact
# records) -- is C64 bound by VALU issue?  Two passes of <= 8 SQ counters.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
for pass in 1 2; do
  if [ $pass = 1 ]; then C=$P1; else C=$P2; fi
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex rx_kernel -d gpurun_out/r05m/c64_p$pass -o run --output-format csv -- python3 bench.py --only c64 --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --no-place --settle 0.3 --no-live-pmc --no-e2e > gpurun_out/r05m/c64_p$pass.log 2>&1
  rc=$?; echo "sq c64 pass $pass rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/sq_summary.py gpurun_out/r05m/c64_p1 gpurun_out/r05m/c64_p2 > gpurun_out/r05m/summary.jsonl
cat gpurun_out/r05m/summary.jsonl
