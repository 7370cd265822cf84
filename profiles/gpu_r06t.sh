# Round 6, call T: Lb's sigma row inside the dW loop (DEN_HB_SIGMA_IN_DW) vs the product, ABBA order
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden.so
B=$PWD/deblur-e-nerf_amd/libden_sigdw.so
bash profiles/ab.sh r06t 1 $B $A
bash profiles/ab.sh r06t 1 $A $B
bash profiles/ab.sh r06t 1 $B $A
bash profiles/ab.sh r06t 1 $A $B
