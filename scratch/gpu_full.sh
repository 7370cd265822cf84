mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/full.log 2>&1
echo "suite rc=$?"
grep -E "passed|failed" gpurun_out/full.log | tail -2
