#!/bin/bash
# Round-2 evidence, one box, one tree (profiles/r02):
#  * GPU suite + smoke;
#  * the default bench command itself under rocprofv3 kernel tracing (every
#    kernel's average duration beside the bench line it produced);
#  * FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md) of
#    the C1500 / C64 / CMIX rx kernels on the same box.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
step gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_prof 900 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py
for c in c1500 c64 cmix; do
  step fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d $O/fetch_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
  step write_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d $O/write_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
done
python tools/pmc_summary.py $O/pmc_summary.json c1500=$O/fetch_c1500,$O/write_c1500,$O/stats c64=$O/fetch_c64,$O/write_c64 cmix=$O/fetch_cmix,$O/write_cmix > $O/pmc_summary.log 2>&1
cat gpurun_out/steps.log
