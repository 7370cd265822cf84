# Round 4, call N: the product build against a -fno-slp-vectorize build (no v_pk_add_f32 in the forward epilogue), A B A B
set -e
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
timeout -k 10 200 $B > gpurun_out/r04n_a1.log 2>&1
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_noslp.so timeout -k 10 200 $B > gpurun_out/r04n_b1.log 2>&1
timeout -k 10 200 $B > gpurun_out/r04n_a2.log 2>&1
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_noslp.so timeout -k 10 200 $B > gpurun_out/r04n_b2.log 2>&1
echo done
