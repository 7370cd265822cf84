# Round 2, call L: final check after the pixel-bandwidth forward and templated dW changes
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/l_gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/l_smoke.log 2>&1
timeout -k 10 420 python bench.py --steps 20 --warmup 3 > gpurun_out/l_bench.log 2>&1
timeout -k 10 300 python profiles/bench_ziggy.py --opt-steps 4 --warmup 1 > gpurun_out/l_ziggy.log 2>&1
timeout -k 10 200 python profiles/ngp_bench.py > gpurun_out/l_ngp_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l_prof_ziggy -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/l_prof_ziggy.log 2>&1
