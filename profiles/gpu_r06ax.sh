# Round 6, call AX: kernel trace of a short default-config bench run: GPU idle between the step's kernels
set -e
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06ax_trace -o r06ax -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r06ax_bench.json 2> gpurun_out/r06ax_bench.err
f=$(find gpurun_out/r06ax_trace -name "*kernel_trace.csv" | head -1)
python3 profiles/step_gaps.py $f > gpurun_out/r06ax_gaps.jsonl
rm -f $f
tail -4 gpurun_out/r06ax_gaps.jsonl
