# Round 4, call F: the GPU suite and smoke on the pruned tree
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --maxfail 6 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04f_tests.log 2>&1 || true
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1
echo done
