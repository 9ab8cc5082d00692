#!/bin/bash
# A/B full vs compact records; refreshed rocprof evidence for profiles/r01.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step ab_c1500 300 python tools/ab.py c1500 3:33 3:33:c 3:32:c 3:1:c 3:32
step ab_c64 300 python tools/ab.py c64 0:32 0:32:c 0:0:c 0:0
for c in c1500 c64 cmix; do
  step stats_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats_$c -o run --output-format csv -- python bench.py --only $c --steps 20 --no-cpu --no-check --no-membench --no-rec32
  step fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d gpurun_out/prof/fetch_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
  step write_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d gpurun_out/prof/write_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
done
python tools/pmc_summary.py gpurun_out/prof/pmc_summary.json c1500=gpurun_out/prof/fetch_c1500,gpurun_out/prof/write_c1500,gpurun_out/prof/stats_c1500 c64=gpurun_out/prof/fetch_c64,gpurun_out/prof/write_c64,gpurun_out/prof/stats_c64 cmix=gpurun_out/prof/fetch_cmix,gpurun_out/prof/write_cmix,gpurun_out/prof/stats_cmix > gpurun_out/pmc_summary.log 2>&1
cat gpurun_out/steps.log
