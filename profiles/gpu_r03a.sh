# Round 3, call A: the ray / timestamp gradient chain (tau_r through the camera pose), the ngp
# zero-gradient scatter fix, alpha compositing, and the rest of the GPU suite
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_raygrad_gpu.py tests/test_deblur_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/a_raygrad.log 2>&1
rc1=$?
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect tests/test_raygrad_gpu.py --deselect tests/test_deblur_gpu.py > gpurun_out/a_gpu_tests.log 2>&1
rc2=$?
echo "raygrad+deblur rc=$rc1 suite rc=$rc2"
tail -5 gpurun_out/a_raygrad.log gpurun_out/a_gpu_tests.log
