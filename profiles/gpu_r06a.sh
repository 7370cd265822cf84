# Round 6 (a): the evaluation hooks / PosedImage / SSIM tests first, then the whole GPU suite and smoke()
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eval_epoch_gpu.py tests/test_eval_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/r06a_eval_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06a_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r06a_gpu_tests.log 2>&1
echo done
