mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_eval_gpu.py tests/test_render_gpu.py -k "eval or metric or fixed_sampler" -v -s --timeout 120 --timeout-method thread > gpurun_out/d_eval.log 2>&1
echo "eval rc=$?"
timeout -k 10 400 python -u bench.py --psnr-only --psnr-steps 2000 > gpurun_out/d_psnr.log 2>&1
echo "psnr rc=$?"
tail -2 gpurun_out/d_psnr.log
