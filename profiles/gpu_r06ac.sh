# Round 6, call AC: the 12-slot rows (libden.so: + dz_b, bottleneck, G) vs 10-slot rows (+ dz_b only,
# bottleneck and G contiguous) and both with a workgroup-dependent start in the hidden launches
# (DEN_HB_ROTATE), each build once in each position of a 4-run group
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
A=$D/libden.so; B=$D/libden_rows10.so; C=$D/libden_rows10rot.so; E=$D/libden_rows12rot.so
bash profiles/ab.sh r06ac 1 $A $B $C $E
bash profiles/ab.sh r06ac 1 $B $C $E $A
bash profiles/ab.sh r06ac 1 $C $E $A $B
bash profiles/ab.sh r06ac 1 $E $A $B $C
