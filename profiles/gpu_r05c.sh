#!/bin/bash
# r05c: dataset build-path parity tests (den_queue_raw_events & co.); PSNR leg: 8 batch sequences of the
# chosen leg, HIP F32 + BF16; the oracle (torch's own GPU kernels, not libden) trained on the same 8
# sequences for its own sequence-to-sequence spread
set -o pipefail
mkdir -p gpurun_out/psnr_oracle_gpu
timeout -k 10 300 python -u -m pytest tests/test_dataset_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05c_dataset_tests.log 2>&1 || exit $?
timeout -k 10 420 python -u profiles/psnr_sweep.py --seqs 8 --modes f32,bf16 --out gpurun_out/r05c_psnr_sweep.jsonl --variants '[{}]' > gpurun_out/r05c_psnr.log 2>&1 || exit $?
for k in 0 1 2 3 4 5 6 7; do
  timeout -k 10 240 python -u tests/golden/make_psnr_oracle.py --seq $k --device cuda --out-dir gpurun_out/psnr_oracle_gpu >> gpurun_out/r05c_oracle_gpu.log 2>&1 || exit $?
done
