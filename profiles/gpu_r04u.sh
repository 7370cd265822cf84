# Round 4, call U: the forward with scalar DMA offsets / m0 and the bias table at LDS offset 0 (the
# product build now) -- GPU suite and smoke on it; A/B against the previous forward (libden_old.so,
# den_render.hip of 9204383) A B A B on this box; the default bench line; the N-rank path rehearsed
# over gloo on the shared GPU; the converged-PSNR seed study
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04u_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04u_smoke.log 2>&1
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
V=$PWD/deblur-e-nerf_amd/libden_old.so
timeout -k 10 200 $B > gpurun_out/r04u_a1.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04u_b1.log 2>&1
timeout -k 10 200 $B > gpurun_out/r04u_a2.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04u_b2.log 2>&1
S=$(date +%s)
timeout -k 10 400 python bench.py > gpurun_out/r04u_bench.log 2>&1
echo "bench_wall_s $(( $(date +%s) - S ))" >> gpurun_out/r04u_bench.log
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-extra-legs --psnr-steps 0 > gpurun_out/r04u_n2.log 2>&1
timeout -k 10 500 python -u profiles/psnr_seeds.py --seeds 8 > gpurun_out/r04u_psnr_seeds.log 2>&1
echo done
