# Round 4, call C: the persistent forward (continuous weight ring across 256-sample items) and the
# pruned build variants: debug render check, the whole GPU suite, then the bench line for timing
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python profiles/dbg_persist.py > gpurun_out/dbg_persist.log 2>&1
timeout -k 10 900 python -u -m pytest -q --maxfail 6 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04c_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-legs --psnr-steps 0 > gpurun_out/r04c_bench.log 2>&1
echo done
