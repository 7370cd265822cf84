mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nerfacc_gpu.py tests/test_deblur_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1
