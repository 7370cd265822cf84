# A/B: the committed build (libden_base.so) against the working tree's libden.so, alternated on one box
set -e
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-legs --psnr-steps 0 --no-gemm-peak"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_train_gpu.py > gpurun_out/ab_tests.log 2>&1
for r in 1 2; do
  DEN_LIB=deblur-e-nerf_amd/libden_base.so timeout -k 10 300 $B > gpurun_out/ab_base$r.log 2>&1
  timeout -k 10 300 $B > gpurun_out/ab_new$r.log 2>&1
done
