# ngp MFMA kernels: parity (incl. ragged tiles / odd level counts), then kernel-trace profiles of the
# ngp_bench and configs[3] emulation
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_mf2.log 2>&1 || echo PARITY_FAIL >> gpurun_out/tngp_mf2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ziggy -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/prof_ziggy.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ngp -o run -- python profiles/ngp_bench.py --iters 5 > gpurun_out/prof_ngp.log 2>&1
