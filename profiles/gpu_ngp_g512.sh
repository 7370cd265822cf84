# grid cap 512 default: ngp parity, ngp_bench, configs[3] emulation
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py tests/test_nerfacc_gpu.py -v -q --timeout 120 --timeout-method thread > gpurun_out/tg512.log 2>&1
timeout -k 10 200 python profiles/ngp_bench.py > gpurun_out/g512_ngp.log 2>&1
timeout -k 10 300 python profiles/bench_ziggy.py --opt-steps 4 --warmup 1 > gpurun_out/g512_ziggy.log 2>&1
