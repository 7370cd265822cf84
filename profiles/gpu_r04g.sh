# Round 4, call G: configs[3] per-rank emulation (profiles/bench_ziggy.py) on the r04 tree, plain
# timing and a kernel-trace summary
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python profiles/bench_ziggy.py --opt-steps 4 --warmup 1 > gpurun_out/r04g_ziggy.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04g_prof_ziggy -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/r04g_prof_ziggy.log 2>&1
echo done
