# Round 6 (g): the default bench.py line as the driver runs it (now with the 128-sample BF16 - F32 PSNR leg)
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
START=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r06g_bench_default.json 2> gpurun_out/r06g_bench_default.err
echo "wall_s $(( $(date +%s) - START ))" >> gpurun_out/r06g_bench_default.err
echo done
