# Round 4, call M: timing-only S0R variants (x1: no softplus, x2: no S'_0 compute) beside the product build
set -e
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
timeout -k 10 200 $B > gpurun_out/r04m_base.log 2>&1
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_x1.so timeout -k 10 200 $B > gpurun_out/r04m_x1.log 2>&1
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_x2.so timeout -k 10 200 $B > gpurun_out/r04m_x2.log 2>&1
echo done
