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
# the PMC passes run the kernel shape the traced bench chose for each config
# (PPTK_RX_VARIANT; results never change), so counters and trace agree
variant() {
  python - "$1" <<'PY'
import json, sys
from pptk_amd.rx import VARIANTS
line = next(l for l in open("gpurun_out/bench_prof.log") if l.startswith("{"))
d = json.loads(line)
v = d["roofline"]["kernel_variant"] if sys.argv[1] == "c1500" else \
    d["secondary"][sys.argv[1]]["kernel_variant"]
print(VARIANTS.index(v))
PY
}
for c in c1500 c64 cmix; do
  export PPTK_RX_VARIANT=$(variant $c)
  echo "$c PPTK_RX_VARIANT=$PPTK_RX_VARIANT" >> gpurun_out/steps.log
  step fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d $O/fetch_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
  step write_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d $O/write_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3
done
unset PPTK_RX_VARIANT
python tools/pmc_summary.py $O/pmc_summary.json c1500=$O/fetch_c1500,$O/write_c1500,$O/stats c64=$O/fetch_c64,$O/write_c64 cmix=$O/fetch_cmix,$O/write_cmix > $O/pmc_summary.log 2>&1
cat gpurun_out/steps.log
