#!/bin/bash
# r05as: head backward Lg weight gradient as 2 x 2 output tiles per wave over a shared bottleneck-tile buffer: phase profile, GPU suite, bench
set -o pipefail
mkdir -p gpurun_out
DEN_LIB=deblur-e-nerf_amd/libden_hprof.so timeout -k 10 240 python -u profiles/head_prof.py > gpurun_out/r05as_head_prof.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05as_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05as_bench.json 2> gpurun_out/r05as_bench.err
