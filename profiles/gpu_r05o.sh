#!/bin/bash
# r05o: the streamed weight-gradient launch alone vs inside the step (profiles/dws_micro.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u profiles/dws_micro.py > gpurun_out/r05o_base.log 2>&1 || exit $?
DEN_LIB=deblur-e-nerf_amd/libden_dws4.so timeout -k 10 240 python -u profiles/dws_micro.py > gpurun_out/r05o_dws4.log 2>&1
