# Round 6, call W: GPU suite + smoke + default bench line on the tree with block-major rows and the early
# derivative factors
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06w_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r06w_gpu_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r06w_bench_default.json 2> gpurun_out/r06w_bench.err
