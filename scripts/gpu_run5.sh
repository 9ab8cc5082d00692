#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
F=$PWD/build/ab_full/libpptkrx.so
step p_nt 300 python bench.py --only c1500 --steps 30 --no-cpu --no-check
step p_pl 300 env PPTK_RX_TUNE=0 python bench.py --only c1500 --steps 30 --no-cpu --no-check --no-membench
step f_nt 300 env PPTK_RX_LIB=$F python bench.py --only c1500 --steps 30 --no-cpu --no-check --no-membench
step f_pl 300 env PPTK_RX_LIB=$F PPTK_RX_TUNE=0 python bench.py --only c1500 --steps 30 --no-cpu --no-check --no-membench
step p_nt2 300 python bench.py --only c1500 --steps 30 --no-cpu --no-check --no-membench
step p_c64 300 python bench.py --only c64 --steps 30 --no-cpu --no-check --no-membench
step f_c64 300 env PPTK_RX_LIB=$F python bench.py --only c64 --steps 30 --no-cpu --no-check --no-membench
for f in p_nt p_pl f_nt f_pl p_nt2 p_c64 f_c64; do echo "$f $(grep -h 'rank 0' gpurun_out/$f.log | tr '\n' ' ')"; done
