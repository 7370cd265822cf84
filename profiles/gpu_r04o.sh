# Round 4, call O: Lb timing-only variants (lb1: no sigma weight-gradient row, lb2: no sigma dz DMA) beside the product
set -e
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
timeout -k 10 200 $B > gpurun_out/r04o_base.log 2>&1
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_lb1.so timeout -k 10 200 $B > gpurun_out/r04o_lb1.log 2>&1
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_lb2.so timeout -k 10 200 $B > gpurun_out/r04o_lb2.log 2>&1
echo done
