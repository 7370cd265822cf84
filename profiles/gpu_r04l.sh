# Round 4, call L: S'_0 recomputed in the layer-1 hidden launch (S0R) -- the render / train GPU tests,
# then the bench with the forward not storing S'_0 against the same tree storing it (DEN_AB_KEEP_S0)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_train_gpu.py > gpurun_out/r04l_tests.log 2>&1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r04l_bench_s0r.log 2>&1
DEN_AB_KEEP_S0=1 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r04l_bench_keep.log 2>&1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r04l_bench_s0r2.log 2>&1
echo done
