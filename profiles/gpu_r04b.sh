# Round 4, call B: the composed fit_step DDP test (2 processes, gloo, step_ziggy composition)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_fit_ddp_gpu.py > gpurun_out/r04b_tests.log 2>&1
echo done
