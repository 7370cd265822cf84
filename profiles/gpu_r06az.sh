# Round 6, call AZ: per-variant hidden launch times with the pe fold (kernel trace: L7..L2 PEM 0 minus
# L5, L5 PEM 1, L1 PEM 2, Lb)
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06az_prof -o run -- python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r06az_prof.log 2>&1
rm -f gpurun_out/r06az_prof/run_kernel_trace.csv gpurun_out/r06az_prof/run_agent_info.csv
head -8 gpurun_out/r06az_prof/run_kernel_stats.csv
