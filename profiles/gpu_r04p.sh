# Round 4, call P: sigma's weight-gradient row of Lb from the dW loop's own S7 operands -- render / train /
# deblur GPU tests, then two bench runs
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_train_gpu.py tests/test_deblur_gpu.py tests/test_dp_gpu.py > gpurun_out/r04p_tests.log 2>&1
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
timeout -k 10 200 $B > gpurun_out/r04p_b1.log 2>&1
timeout -k 10 200 $B > gpurun_out/r04p_b2.log 2>&1
echo done
