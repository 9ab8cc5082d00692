#!/bin/bash
# Full validation + bench + rocprof evidence (profiles/r01), one box.
# The headline line (C1500) is measured by the very command rocprofv3 traces
# (bench_prof_c1500: roofline, cpu_baseline, parity checks all included), so
# its kernel_ms and the rocprof average for the chosen kernel variant come from
# the same launches. The unprofiled full bench (all configs) follows.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests -x -q -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_prof_c1500 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats_c1500 -o run --output-format csv -- python bench.py --only c1500 --steps 20 --warmup 3 --cpu-seconds 10 --no-rec32
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
for c in c64 cmix; do
  step stats_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats_$c -o run --output-format csv -- python bench.py --only $c --steps 20 --no-cpu --no-check --no-membench --no-rec32
done
for c in c1500 c64 cmix; do
  step fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d gpurun_out/prof/fetch_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
  step write_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d gpurun_out/prof/write_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
done
python tools/pmc_summary.py gpurun_out/prof/pmc_summary.json c1500=gpurun_out/prof/fetch_c1500,gpurun_out/prof/write_c1500,gpurun_out/prof/stats_c1500 c64=gpurun_out/prof/fetch_c64,gpurun_out/prof/write_c64,gpurun_out/prof/stats_c64 cmix=gpurun_out/prof/fetch_cmix,gpurun_out/prof/write_cmix,gpurun_out/prof/stats_cmix > gpurun_out/pmc_summary.log 2>&1
cat gpurun_out/steps.log
