#!/bin/bash
# Round 6 tree: the default bench under rocprofv3 kernel
# tracing with ROCTx ranges (PPTK_BENCH_ROCTX=1, --kernel-rename: the timed
# launches of every config are reported under "timed_<cfg>" in
# kernel_stats.csv, apart from the placement probes, autotune trials and
# settle launches of the same kernels), then FETCH_SIZE / WRITE_SIZE passes
# (separate runs, MI355X_MICROARCH.md) of every config's rx kernel and of
# the three rate-limiter runs, summarised into $O/pmc_summary.json.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06prof3
mkdir -p $O
export PPTK_BENCH_ROCTX=1
step bench_prof 900 rocprofv3 --kernel-trace --marker-trace --kernel-rename --stats -d $O/stats -o run --output-format csv -- python bench.py --no-live-pmc --detail $O/bench_prof_detail.json || exit $?
unset PPTK_BENCH_ROCTX
grep '^{' $O/bench_prof.log | tail -1 > $O/bench_prof.json
variant() {
  python - "$1" <<'PY'
import json, sys
from pptk_amd.rx import VARIANTS
d = json.loads(open("gpurun_out/r06prof3/bench_prof.json").read())
print(VARIANTS.index(d["configs"][sys.argv[1]]["variant"]))
PY
}
for c in c1500 c64 cmix imix jmix; do
  export PPTK_RX_VARIANT=$(variant $c)
  echo "$c PPTK_RX_VARIANT=$PPTK_RX_VARIANT" >> $O/steps.log
  step fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d $O/fetch_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3 --no-live-pmc || exit $?
  step write_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d $O/write_$c -o run --output-format csv -- python bench.py --only $c --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0.3 --no-live-pmc || exit $?
done
unset PPTK_RX_VARIANT
for op in permit_records permit_keys permit_keys_denying; do
  step fetch_$op 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$op -o run --output-format csv -- python tools/opbench.py $op || exit $?
  step write_$op 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_$op -o run --output-format csv -- python tools/opbench.py $op || exit $?
done
N=16777216
python tools/pmc_summary.py $O/pmc_summary.json c1500=$O/fetch_c1500,$O/write_c1500,$O/stats c64=$O/fetch_c64,$O/write_c64,$O/stats cmix=$O/fetch_cmix,$O/write_cmix,$O/stats imix=$O/fetch_imix,$O/write_imix,$O/stats jmix=$O/fetch_jmix,$O/write_jmix,$O/stats \
  "op:permit_records:permit_|rocprim:$N:7=$O/fetch_permit_records,$O/write_permit_records" \
  "op:permit_keys:permit_|rocprim:$N:7=$O/fetch_permit_keys,$O/write_permit_keys" \
  "op:permit_keys_denying:permit_|rocprim:$N:7=$O/fetch_permit_keys_denying,$O/write_permit_keys_denying" > $O/pmc_summary.log 2>&1
cat $O/steps.log
grep -A3 '"timed_range' $O/pmc_summary.json | head -20
