# ngp dW split reduction parallel over splits: parity, then a kernel trace of the configs[3] emulation
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_red.log 2>&1 || echo PARITY_FAIL >> gpurun_out/tngp_red.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/red_prof -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/red_prof.log 2>&1
timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 3 --warmup 1 > gpurun_out/red_ziggy.log 2>&1
