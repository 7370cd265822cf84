# Round 6, call BH: the whole GPU suite (incl. tests/test_pe_fold_gpu.py) and smoke on the final tree
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06bh_gpu_tests.log 2>&1
tail -1 gpurun_out/r06bh_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r06bh_gpu_tests.log 2>&1
tail -1 gpurun_out/r06bh_gpu_tests.log
