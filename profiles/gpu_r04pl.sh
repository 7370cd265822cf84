# Round 4, call PL: instruction-fetch counters for two placements of the same code -- the product (every hot
# kernel page-aligned) and the r04u build (libden_unal.so, render_bwd_kernel at 0x1c2900) -- plus a timed
# bench of each on the same box
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
P="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
V=$PWD/deblur-e-nerf_amd/libden_unal.so
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
C=$(python profiles/pick_counters.py gpurun_out/counters.txt SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH GRBM_GUI_ACTIVE)
echo "pmc: $C" > gpurun_out/r04pl_sets.txt
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r04pl_al -o run -- $P > gpurun_out/r04pl_al.log 2>&1
DEN_LIB=$V timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r04pl_un -o run -- $P > gpurun_out/r04pl_un.log 2>&1
timeout -k 10 200 $B > gpurun_out/r04pl_t_al.log 2>&1
DEN_LIB=$V timeout -k 10 200 $B > gpurun_out/r04pl_t_un.log 2>&1
echo done
