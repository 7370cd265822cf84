# quick GPU iteration: parity tests, then one bench line per configuration (profiles/gpu_round.sh adds the rocprof passes)
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/tq.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bq.log 2>&1
timeout -k 10 300 python bench.py --pixbw --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bqp.log 2>&1
