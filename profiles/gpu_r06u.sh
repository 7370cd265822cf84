# Round 6, call U: the position effect (r06t: the second bench process of a pair runs the hidden launches
# ~0.2 ms faster whatever the build) controlled: pre-r06n aliasing (base), r06n, block-major rows, each
# build in each position of a 3-run group.
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
bash profiles/ab.sh r06u 1 $D/libden_base.so $D/libden.so $D/libden_rows.so
bash profiles/ab.sh r06u 1 $D/libden_rows.so $D/libden_base.so $D/libden.so
bash profiles/ab.sh r06u 1 $D/libden.so $D/libden_rows.so $D/libden_base.so
bash profiles/ab.sh r06u 1 $D/libden_base.so $D/libden_rows.so $D/libden.so
