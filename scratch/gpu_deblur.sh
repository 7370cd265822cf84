mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_deblur_gpu.py tests/test_raygrad_gpu.py -v -s --timeout 120 --timeout-method thread > gpurun_out/c_deblur.log 2>&1
echo "default rc=$?"
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_precact.so timeout -k 10 200 python -u -m pytest tests/test_deblur_gpu.py -k ngp -v -s --timeout 120 --timeout-method thread > gpurun_out/c_precact.log 2>&1
echo "precact rc=$?"
