#!/bin/bash
# r05al: sigma's dz packed in 1 KiB runs (sigma_dz_offset): GPU suite, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05al_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05al_bench.json 2> gpurun_out/r05al_bench.err
