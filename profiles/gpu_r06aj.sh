# Round 6, call AJ: GPU suite + smoke + default bench line on the final tree (rows with dz_b, sigma-row fence removed)
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06aj_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r06aj_gpu_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r06aj_bench_default.json 2> gpurun_out/r06aj_bench.err
