# Round 6, call AT: Lb at 8 waves too (sigma k-step W^T fragment in LDS, S' fragments read in the
# epilogue, chain prefetch depth 2 or 1) against the product (Lb at 4 waves), each build in each
# position of a 3-run group
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
A=$D/libden.so; B=$D/libden_lb8pf2.so; C=$D/libden_lb8.so
bash profiles/ab.sh r06at 1 $A $B $C
bash profiles/ab.sh r06at 1 $C $A $B
bash profiles/ab.sh r06at 1 $B $C $A
bash profiles/ab.sh r06at 1 $A $C $B
