set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ziggy -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/prof_ziggy.log 2>&1
