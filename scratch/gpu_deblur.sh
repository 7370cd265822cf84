mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_deblur_gpu.py -v -s --timeout 120 --timeout-method thread > gpurun_out/c_deblur.log 2>&1
echo "deblur rc=$?"
grep -E "passed|failed" gpurun_out/c_deblur.log | tail -1
