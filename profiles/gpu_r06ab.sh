# Round 6, call AB: dz_b, the bottleneck and G joined to the block-major rows (head and Lb streams in one
# row).  GPU suite on the new build, then ABBA x 2 against the 9-slot rows build.
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ab_gpu_tests.log 2>&1
A=$PWD/deblur-e-nerf_amd/libden_rows9.so
B=$PWD/deblur-e-nerf_amd/libden.so
bash profiles/ab.sh r06ab 1 $A $B
bash profiles/ab.sh r06ab 1 $B $A
bash profiles/ab.sh r06ab 1 $B $A
bash profiles/ab.sh r06ab 1 $A $B
