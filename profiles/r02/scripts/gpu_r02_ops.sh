#!/bin/bash
# Round-2 evidence for the secondary batch ops (profiles/r02): kernel trace
# and FETCH_SIZE / WRITE_SIZE passes of each op run alone (tools/opbench.py),
# summarized with the write amplification WRITE_SIZE / bytes changed.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
for op in tx rewrite mss permit binned allgather; do
  step stats_$op 300 rocprofv3 --kernel-trace --stats -d $O/stats_$op -o run --output-format csv -- python tools/opbench.py $op --steps 10
  step fetch_$op 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$op -o run --output-format csv -- python tools/opbench.py $op
  step write_$op 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_$op -o run --output-format csv -- python tools/opbench.py $op
done
N=16777216
python tools/pmc_summary.py $O/pmc_ops.json \
  "op:tx:rx_kernel:$((4*N))=$O/fetch_tx,$O/write_tx" \
  "op:rewrite:rx_rewrite_kernel:$((17*N))=$O/fetch_rewrite,$O/write_rewrite" \
  "op:mss:rx_mss_kernel:$((4*N))=$O/fetch_mss,$O/write_mss" \
  "op:permit:permit_|rocprim:$N=$O/fetch_permit,$O/write_permit" \
  "op:binned:bin_|rx_kernel:$((64*N))=$O/fetch_binned,$O/write_binned" \
  "op:allgather:rx_kernel|nccl|rccl|AllGather:$((72*N))=$O/fetch_allgather,$O/write_allgather" > $O/pmc_ops.log 2>&1
cat gpurun_out/steps.log
