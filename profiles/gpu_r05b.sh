#!/bin/bash
# r05b: dataset build-path parity tests (den_queue_raw_events & co.) + PSNR leg: 8 batch sequences of
# the chosen training leg, F32 + BF16, scored on 8 x 32^2 views, and F32 on the round-4 style 4 x 64^2 views
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dataset_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05b_dataset_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u profiles/psnr_sweep.py --seqs 8 --modes f32,bf16 --out gpurun_out/r05b_psnr_sweep.jsonl --variants '[{}]' > gpurun_out/r05b_psnr.log 2>&1 || exit $?
timeout -k 10 300 python -u profiles/psnr_sweep.py --seqs 8 --modes f32 --out gpurun_out/r05b_psnr_sweep.jsonl --variants '[{"view":64,"n_views":4}]' >> gpurun_out/r05b_psnr.log 2>&1
