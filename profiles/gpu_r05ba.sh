#!/bin/bash
# r05ba: the forward cycle split with the item tail divided at the compositing barrier (DEN_FWD_PROF build)
set -o pipefail
mkdir -p gpurun_out
DEN_LIB=deblur-e-nerf_amd/libden_fprof.so timeout -k 10 240 python -u profiles/fwd_prof.py train > gpurun_out/r05ba_fwd_prof.txt 2>&1
