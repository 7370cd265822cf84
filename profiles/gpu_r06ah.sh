# Round 6, call V: Lb sigma row without its leading scheduling fence (DEN_HB_SIGMA_NOFENCE) vs the product, ABBA x 2
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_nofence.so
bash profiles/ab.sh r06ah 1 $A $B
bash profiles/ab.sh r06ah 1 $B $A
bash profiles/ab.sh r06ah 1 $B $A
bash profiles/ab.sh r06ah 1 $A $B
