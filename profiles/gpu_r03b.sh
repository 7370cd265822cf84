# Round 3, call B: ray / timestamp gradients with f32-floored bounds, the step goldens against the
# reference's f64 run (per-call timestamp gradients, tau_r), event-prep backward
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_raygrad_gpu.py tests/test_deblur_gpu.py tests/test_ngp_gpu.py -v -s --timeout 120 --timeout-method thread > gpurun_out/b_raygrad.log 2>&1
echo "rc=$?"
grep -E "PASSED|FAILED|ERROR" gpurun_out/b_raygrad.log | tail -60
