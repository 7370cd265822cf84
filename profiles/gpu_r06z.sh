# Round 6, call V: the dz stores of a block issued after its dW phase (DEN_HB_LATE_STORES) vs the product, ABBA x 2
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_late.so
bash profiles/ab.sh r06z 1 $A $B
bash profiles/ab.sh r06z 1 $B $A
bash profiles/ab.sh r06z 1 $B $A
bash profiles/ab.sh r06z 1 $A $B
