#!/bin/bash
# Round-3 evidence, one box, one tree (profiles/r03):
#  * smoke;
#  * the default bench command under rocprofv3 kernel tracing (its own
#    same-run PMC passes off: no profiler nesting);
#  * FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md) of
#    the C1500 / C64 / CMIX / IMIX / JMIX rx kernels and of the three rate
#    limiter runs alone (tools/opbench.py permit_<run>).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_prof 900 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --no-live-pmc
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
for c in c1500 c64 cmix imix jmix; do
  export PPTK_RX_VARIANT=$(variant $c)
  echo "$c PPTK_RX_VARIANT=$PPTK_RX_VARIANT" >> gpurun_out/steps.log
  step fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d $O/fetch_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3 --no-live-pmc
  step write_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d $O/write_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3 --no-live-pmc
done
unset PPTK_RX_VARIANT
for op in permit_records permit_keys permit_keys_denying; do
  step fetch_$op 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$op -o run --output-format csv -- python tools/opbench.py $op
  step write_$op 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_$op -o run --output-format csv -- python tools/opbench.py $op
done
N=16777216
python tools/pmc_summary.py $O/pmc_summary.json c1500=$O/fetch_c1500,$O/write_c1500,$O/stats c64=$O/fetch_c64,$O/write_c64 cmix=$O/fetch_cmix,$O/write_cmix imix=$O/fetch_imix,$O/write_imix jmix=$O/fetch_jmix,$O/write_jmix \
  "op:permit_records:permit_|rocprim:$N:7=$O/fetch_permit_records,$O/write_permit_records" \
  "op:permit_keys:permit_|rocprim:$N:7=$O/fetch_permit_keys,$O/write_permit_keys" \
  "op:permit_keys_denying:permit_|rocprim:$N:7=$O/fetch_permit_keys_denying,$O/write_permit_keys_denying" > $O/pmc_summary.log 2>&1
cat gpurun_out/steps.log
