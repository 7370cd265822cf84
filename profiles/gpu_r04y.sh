# Round 4, call Y: every hot kernel page-aligned (render_fwd, hidden_bwd x2, dwstream x2, render_bwd;
# DEN_PAGE_ALIGN_ALL, libden_pal.so) against the product (render_bwd aligned only), A P A P on one box
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
V=$PWD/deblur-e-nerf_amd/libden_pal.so
timeout -k 10 200 $B > gpurun_out/r04y_a1.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04y_p1.log 2>&1
timeout -k 10 200 $B > gpurun_out/r04y_a2.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04y_p2.log 2>&1
echo done
