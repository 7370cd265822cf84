# Round 5, call PL: instruction-fetch counters (SQC_ICACHE_*, SQ_IFETCH) for the page-aligned product and the default placement (libden_unal.so, -DDEN_NO_CODE_ALIGN) -- VERDICT r04 item 5 -- plus a timed bench of each on the same box
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
V=$PWD/deblur-e-nerf_amd/libden_unal.so
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
C=$(python profiles/pick_counters.py gpurun_out/counters.txt SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH GRBM_GUI_ACTIVE)
echo "pmc: $C" > gpurun_out/r05pl_sets.txt
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r05pl_al -o run -- $P > gpurun_out/r05pl_al.log 2>&1
DEN_LIB=$V timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r05pl_un -o run -- $P > gpurun_out/r05pl_un.log 2>&1
timeout -k 10 200 $B > gpurun_out/r05pl_t_al.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r05pl_t_un.log 2>&1
echo done
