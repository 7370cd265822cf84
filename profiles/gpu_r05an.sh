#!/bin/bash
# r05an: Lb sigma weight-gradient MFMAs inside the dW stream (rotated column tiles): GPU suite, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05an_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05an_bench.json 2> gpurun_out/r05an_bench.err
