#!/bin/bash
# r05x: the default bench.py line (the driver's N = 1 run: CPU baseline, extra legs, 8-sequence PSNR leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r05x_bench.json 2> gpurun_out/r05x_bench.err
