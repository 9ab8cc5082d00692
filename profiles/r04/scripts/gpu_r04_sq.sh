#!/bin/bash
# Round 4 (VERDICT ask 2): SQ counters of the CMIX launch, T16S6 and M6,
# plus C1500 (T32S3) for comparison -- two passes of <= 8 SQ counters each.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
for spec in cmix:3 cmix:13 cmix:14 c1500:4; do
  cfg=${spec%%:*}; var=${spec##*:}
  for pass in 1 2; do
    if [ $pass = 1 ]; then C=$P1; else C=$P2; fi
    PPTK_RX_VARIANT=$var timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex rx_kernel -d gpurun_out/sq/${cfg}_v${var}_p$pass -o run --output-format csv -- python3 bench.py --only $cfg --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --no-place --settle 0.3 --no-live-pmc > gpurun_out/sq/${cfg}_v${var}_p$pass.log 2>&1
    rc=$?; echo "sq $cfg v$var pass $pass rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/sq_summary.py gpurun_out/sq/*_p1 gpurun_out/sq/*_p2 > gpurun_out/sq/summary.jsonl
cat gpurun_out/sq/summary.jsonl | cut -c1-400
