# Round 6, call V: the L7..L1 epilogue's activation-derivative factors computed in the chain MFMAs' shadow
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_dearly.so
bash profiles/ab.sh r06v 1 $A $B
bash profiles/ab.sh r06v 1 $B $A
bash profiles/ab.sh r06v 1 $B $A
bash profiles/ab.sh r06v 1 $A $B
