# Round 6, call V: pe joins the block-major rows (slot 10, 4 KiB) vs the product, ABBA x 2
# (DEN_HB_DERIV_EARLY) vs the product (block-major rows), ABBA x 2
set -e
set -o pipefail
mkdir -p gpurun_out
A=$PWD/deblur-e-nerf_amd/libden_rows10.so
B=$PWD/deblur-e-nerf_amd/libden_rowspe.so
bash profiles/ab.sh r06ag 1 $A $B
bash profiles/ab.sh r06ag 1 $B $A
bash profiles/ab.sh r06ag 1 $B $A
bash profiles/ab.sh r06ag 1 $A $B
