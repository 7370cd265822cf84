# Round 6, call BB: the pe-fold parity test (folded vs streamed parameter gradients)
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pe_fold_gpu.py -m gpu -v -s --timeout 120 --timeout-method thread > gpurun_out/r06bb_pe_fold.log 2>&1
grep -E "folded vs|passed|failed" gpurun_out/r06bb_pe_fold.log
