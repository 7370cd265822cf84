# Round 4, call J: smoke + the GPU suite on the ABI-4 build
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04j_smoke.log 2>&1
timeout -k 10 900 python -u -m pytest -q --maxfail 6 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04j_tests.log 2>&1
echo done
