#!/bin/bash
# r05i: pixbw BF16 conditioning vs camera speed; the GPU-executed oracle's seed study (8 sequences)
set -o pipefail
mkdir -p gpurun_out/psnr_oracle_gpu
timeout -k 10 300 python -u profiles/probe_pixbw_bf16.py 20,50,200 0 > gpurun_out/r05i_pixbw_probe.log 2>&1 || exit $?
for k in 0 1 2 3 4 5 6 7; do
  timeout -k 10 240 python -u tests/golden/make_psnr_oracle.py --seq $k --device cuda --out-dir gpurun_out/psnr_oracle_gpu >> gpurun_out/r05i_oracle_gpu.log 2>&1 || exit $?
done
