#!/bin/bash
# r05bc: head backward Lr^T with the dz_r transposed fragments read once per item: phase profile, GPU suite, bench
set -o pipefail
mkdir -p gpurun_out
DEN_LIB=deblur-e-nerf_amd/libden_hprof.so timeout -k 10 240 python -u profiles/head_prof.py > gpurun_out/r05bc_head_prof.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05bc_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05bc_bench.json 2> gpurun_out/r05bc_bench.err
