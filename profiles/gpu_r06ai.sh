# Round 6, call V: L7..L1 epilogue without its per-tile scheduling fence (DEN_HB_EPI_NOFENCE) vs the product, ABBA x 2
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_epinf.so
bash profiles/ab.sh r06ai 1 $A $B
bash profiles/ab.sh r06ai 1 $B $A
bash profiles/ab.sh r06ai 1 $B $A
bash profiles/ab.sh r06ai 1 $A $B
