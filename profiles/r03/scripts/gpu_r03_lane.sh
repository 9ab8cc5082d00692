#!/bin/bash
# (the PPTK_RX_LANE_UNROLL2 / PPTK_RX_LANE_WAVES variant was measured and removed from the source: DESIGN.md section 10)
# Round 3: C64 lane kernel -- register sets used in turn (no copy of the
# prefetch registers, no vmcnt(0) per tile) at 3 waves/SIMD (abl/libpptkrx_lane3.so
# = make abvariant NAME=lane3 DEFS="-DPPTK_RX_LANE_UNROLL2 -DPPTK_RX_LANE_WAVES=3")
# against the product (copy, 4 waves/SIMD); in-process A/B, placed buffers.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS=lane3=abl/libpptkrx_lane3.so AB_PLACE=1
timeout -k 10 300 python -u tools/ab.py c64 12:-1 lane3:12:-1 12:-1:c lane3:12:-1:c > gpurun_out/lane_ab.json 2> gpurun_out/lane_ab.log
rc=$?; echo "c64 rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/lane_ab.json')); print({k:v for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
exit $rc
