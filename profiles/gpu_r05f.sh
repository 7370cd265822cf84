#!/bin/bash
# r05f: pe / ve recomputed (dwstream) + the persistent head backward with the Lg weight gradient fused:
# GPU suite, bench line, then the PSNR sequences and the GPU-executed oracle
set -o pipefail
mkdir -p gpurun_out/psnr_oracle_gpu
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05f_bench.json 2> gpurun_out/r05f_bench.err || exit $?
timeout -k 10 420 python -u profiles/psnr_sweep.py --seqs 8 --modes f32,bf16 --out gpurun_out/r05f_psnr_sweep.jsonl --variants '[{}]' > gpurun_out/r05f_psnr.log 2>&1 || exit $?
for k in 0 1 2 3 4 5 6 7; do
  timeout -k 10 240 python -u tests/golden/make_psnr_oracle.py --seq $k --device cuda --out-dir gpurun_out/psnr_oracle_gpu >> gpurun_out/r05f_oracle_gpu.log 2>&1 || exit $?
done
