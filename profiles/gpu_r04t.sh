# Round 4, call T: scalar DMA offsets / m0 in the forward weight stream (DEN_FWD_M0S: no per-piece
# v_readfirstlane; -1.7 % issue cycles per wave-item by profiles/fwd_issue_budget.py) vs the product
# build, A B A B on one box; the variant's forward parity tests first
# plus the bias table at LDS offset 0 (DEN_FWD_BIAS0: bias reads by immediate offsets); both: -2.7 % issue
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/deblur-e-nerf_amd/libden_mb.so
DEN_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_train_gpu.py > gpurun_out/r04t_variant_tests.log 2>&1
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
timeout -k 10 200 $B > gpurun_out/r04t_a1.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04t_b1.log 2>&1
timeout -k 10 200 $B > gpurun_out/r04t_a2.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04t_b2.log 2>&1
echo done
