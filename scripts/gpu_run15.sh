#!/bin/bash
# C64 SipHash A/B (32-bit halves vs uint64 adds), CMIX cost breakdown with
# diagnostic tune bits (8: no record stores, 16: no lane phase).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
export AB_LIBS=old=build/ab_old/libpptkrx.so,sip64=build/ab_sip64/libpptkrx.so
step ab_c64 300 python tools/ab.py c64 0:0 sip64:0:0 old:0:0 0:8 0:16 0:24
step ab_cmix_id 300 python tools/ab.py cmix 3:33 old:3:33 3:41 3:49 3:57 3:0
step ab_cmix_mixed 300 env AB_MIXED=1 AB_LIBS= python tools/ab.py cmix -1:33 -1:49 -1:0 -1:16
step ab_c1500 300 python tools/ab.py c1500 3:33 old:3:33 3:49 3:41
cat gpurun_out/steps.log
