#!/bin/bash
# r05av: dz_b as 8-tile blocks + a sigma array on the layer-major path: phase profile, GPU suite, bench
set -o pipefail
mkdir -p gpurun_out
DEN_LIB=deblur-e-nerf_amd/libden_hprof.so timeout -k 10 240 python -u profiles/head_prof.py > gpurun_out/r05av_head_prof.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05av_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05av_bench.json 2> gpurun_out/r05av_bench.err
