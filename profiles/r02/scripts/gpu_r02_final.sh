#!/bin/bash
# Final-tree evidence of this round (profiles/r02): profiles/r02/scripts/gpu_r02_main.sh
# (GPU suite, smoke, the default bench under kernel tracing, FETCH/WRITE
# passes of the rx kernels) plus the rate limiter's trace and traffic.
bash profiles/r02/scripts/gpu_r02_main.sh || exit $?
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r02p
step stats_permit 300 rocprofv3 --kernel-trace --stats -d $O/stats_permit -o run --output-format csv -- python tools/opbench.py permit --steps 10
step fetch_permit 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_permit -o run --output-format csv -- python tools/opbench.py permit
step write_permit 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_permit -o run --output-format csv -- python tools/opbench.py permit
N=16777216
python tools/pmc_summary.py $O/pmc_ops_permit.json "op:permit:permit_|rocprim:$N=$O/fetch_permit,$O/write_permit" > $O/pmc_ops_permit.log 2>&1
cat gpurun_out/steps.log
