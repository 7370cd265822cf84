# Round 6, call AU: the GPU suite, smoke and the default bench on the 8-wave Lb build
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06au_pytest.log 2>&1
tail -3 gpurun_out/r06au_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06au_smoke.log 2>&1
tail -1 gpurun_out/r06au_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r06au_bench.json 2> gpurun_out/r06au_bench.err
cat gpurun_out/r06au_bench.json
