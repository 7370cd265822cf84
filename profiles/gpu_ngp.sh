# ngp field throughput + kernel-trace summary
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python profiles/ngp_bench.py > gpurun_out/ngp_bench.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ngp -o run -- python profiles/ngp_bench.py --iters 5 > gpurun_out/prof_ngp.log 2>&1
