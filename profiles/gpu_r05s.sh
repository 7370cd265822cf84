#!/bin/bash
# r05s: forward stores pe, the streamed L0 / L5-pe weight gradient reads it (recompute measured slower): GPU suite + bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05s_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05s_bench.json 2> gpurun_out/r05s_bench.err
