# Round 6, call V: L7..L1 with 4 blocks in flight (5-slot ring, 160 KiB) vs 3, ABBA x 2
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_d4.so
bash profiles/ab.sh r06y 1 $A $B
bash profiles/ab.sh r06y 1 $B $A
bash profiles/ab.sh r06y 1 $B $A
bash profiles/ab.sh r06y 1 $A $B
