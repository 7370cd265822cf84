# Round 6, call V: the hidden launches with 8 waves per workgroup (2 per SIMD, 1 row tile each; Lb spills in this build) vs 4 (refactored source), ABBA x 2
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_w8.so
bash profiles/ab.sh r06ar 1 $A $B
bash profiles/ab.sh r06ar 1 $B $A
bash profiles/ab.sh r06ar 1 $B $A
bash profiles/ab.sh r06ar 1 $A $B
