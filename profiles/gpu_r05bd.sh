#!/bin/bash
# r05bd: forward cycle split with and without the per-sample record store (timing-only build NOREC;
# forward alone, inputs unchanged)
set -o pipefail
mkdir -p gpurun_out
for v in fprof fprofnr fprof fprofnr; do
  echo "== $v" >> gpurun_out/r05bd_fwd_prof.txt
  DEN_LIB=deblur-e-nerf_amd/libden_$v.so timeout -k 10 240 python -u profiles/fwd_prof.py train >> gpurun_out/r05bd_fwd_prof.txt 2>&1 || exit $?
done
