#!/bin/bash
# r05n: the r04 tree (commit 67d72bc, its own bench.py and libden built from its sources) and this
# tree back to back on one box: is the streamed L0 / L5-pe weight-gradient launch slower in the r05
# tree, or on this box?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd exp_r04tree && timeout -k 10 240 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0) > gpurun_out/r05n_r04.log 2>&1 || exit $?
DEN_LIB=deblur-e-nerf_amd/libden_dws4.so timeout -k 10 240 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r05n_dws4.log 2>&1 || exit $?
(cd exp_r04tree && timeout -k 10 240 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0) > gpurun_out/r05n_r04b.log 2>&1
