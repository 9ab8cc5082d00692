#!/bin/bash
# Round 5: the kernel timeline of the C8G emulation (copying RCCL stand-in
# beside C1500), unsplit and with the 32-CU split, under rocprofv3 kernel
# tracing: how much of each stand-in kernel ran while an rx kernel ran
# (tools/overlap_trace.py).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ax
mkdir -p $O
step trace_nosplit 400 rocprofv3 --kernel-trace --output-format csv -d $O/nosplit -o run -- python tools/c8g_emul.py 20 --standin 32 --copy || exit $?
step trace_split 400 rocprofv3 --kernel-trace --output-format csv -d $O/split -o run -- python tools/c8g_emul.py 20 --standin 32 --copy --split 32 || exit $?
python3 tools/overlap_trace.py $O/nosplit > $O/overlap_nosplit.json && python3 tools/overlap_trace.py $O/split > $O/overlap_split.json
cat $O/overlap_nosplit.json $O/overlap_split.json
grep -h '^{' $O/trace_nosplit.log $O/trace_split.log | cut -c1-300
