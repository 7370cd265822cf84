# Round 4, call W: is render_bwd_kernel's r04u slowdown (3.11 vs 2.84 ms with byte-identical code) a
# code-placement effect?  The product build against one whose render_bwd_kernel is 4096-byte aligned
# (DEN_RB_ALIGN=4096, libden_rba.so), A C A C on one box
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
V=$PWD/deblur-e-nerf_amd/libden_rba.so
timeout -k 10 200 $B > gpurun_out/r04w_a1.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04w_c1.log 2>&1
timeout -k 10 200 $B > gpurun_out/r04w_a2.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04w_c2.log 2>&1
echo done
