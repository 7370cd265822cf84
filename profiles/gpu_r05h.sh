#!/bin/bash
# r05h: the BF16 backward fault fixed (dwstream fetch inlined): pixbw BF16 probe, GPU suite, bench line,
# PSNR sequences
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u profiles/probe_pixbw_bf16.py > gpurun_out/r05h_pixbw_probe.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05h_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05h_bench.json 2> gpurun_out/r05h_bench.err || exit $?
timeout -k 10 420 python -u profiles/psnr_sweep.py --seqs 8 --modes f32,bf16 --out gpurun_out/r05h_psnr_sweep.jsonl --variants '[{}]' > gpurun_out/r05h_psnr.log 2>&1
