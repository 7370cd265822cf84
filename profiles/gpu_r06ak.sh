# Round 6, call V: the whole library built with -fno-slp-vectorize (no v_pk_*_f32 in the forward epilogue) vs the product, ABBA x 2
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_noslp.so
bash profiles/ab.sh r06ak 1 $A $B
bash profiles/ab.sh r06ak 1 $B $A
bash profiles/ab.sh r06ak 1 $B $A
bash profiles/ab.sh r06ak 1 $A $B
