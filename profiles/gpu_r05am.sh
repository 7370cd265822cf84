#!/bin/bash
# r05am: Lb fetches sigma's dz per 16-block run: GPU suite, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05am_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05am_bench.json 2> gpurun_out/r05am_bench.err
