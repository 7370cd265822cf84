# Round 3, call C: smoke, the default bench line (configs[1] + configs[2] / F32 legs, CPU baseline,
# PSNR legs), the rocprofv3 kernel-trace summary of the bench and the FETCH / WRITE PMC passes
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c_smoke.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r03c_bench.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r03c_prof.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03c_pmc_fetch -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r03c_pmc_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03c_pmc_write -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r03c_pmc_write.log 2>&1
