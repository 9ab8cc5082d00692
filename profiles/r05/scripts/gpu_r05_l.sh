#!/bin/bash
# Round 5: direct global->LDS loads (global_load_lds_dwordx4) against vector
# loads on C1500-shaped tiles, read-only and with the 4 KB record run per
# tile, interleaved in one process (tools/glds_probe.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05l
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/glds_probe.py --out gpurun_out/r05l/glds_probe.json > gpurun_out/r05l/glds_probe.log 2>&1
rc=$?; echo "glds_probe rc=$rc"
python3 -c "
import json; d=json.load(open('gpurun_out/r05l/glds_probe.json'))
for k, v in d['results'].items(): print(f'{k:28s} {v[\"ms\"]:8.4f} ms {v[\"read_gbs\"]:8.1f} GB/s')" || true
exit $rc
