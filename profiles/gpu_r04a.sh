# Round 4, call A: the GPU parity tests this round changed (step goldens with the cone-angle grid
# replay, masked TV / per-ray background checks, the cone ngp fixture, tighter BF16 bounds, eval)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_deblur_gpu.py tests/test_ngp_gpu.py tests/test_eval_gpu.py tests/test_train_gpu.py > gpurun_out/r04a_tests.log 2>&1
echo done
