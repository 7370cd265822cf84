# Round 2, call J: the full GPU suite, smoke, the headline bench, and kernel-trace summaries of the
# ngp field (ngp_bench) and the configs[3] emulation after the MFMA field / quad scatter / wave march /
# segment-parallel pixel-bandwidth work; FETCH / WRITE passes of ngp_bench.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/j_gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/j_smoke.log 2>&1
timeout -k 10 420 python bench.py --steps 20 --warmup 3 > gpurun_out/j_bench.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/j_prof_ngp -o run -- python profiles/ngp_bench.py --iters 5 > gpurun_out/j_prof_ngp.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/j_prof_ziggy -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/j_prof_ziggy.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/j_pmc_fetch -o run -- python profiles/ngp_bench.py --iters 2 > gpurun_out/j_pmc_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/j_pmc_write -o run -- python profiles/ngp_bench.py --iters 2 > gpurun_out/j_pmc_write.log 2>&1
