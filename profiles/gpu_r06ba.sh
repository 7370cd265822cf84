# Round 6, call BA: L1's folded launch two blocks ahead (dz_0 staged over the wave's own dz_1 tile after a
# mid-block barrier, 6 W^T k-steps in LDS; b: two S' fragments in flight and LDS W^T read at use) against
# the product (one block ahead, separate stages): GPU suite on a, then the A/B in all positions
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
DEN_LIB=$D/libden_pe2d2a.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ba_pytest.log 2>&1
tail -1 gpurun_out/r06ba_pytest.log
A=$D/libden.so; B=$D/libden_pe2d2a.so; C=$D/libden_pe2d2b.so
bash profiles/ab.sh r06ba 1 $A $B $C
bash profiles/ab.sh r06ba 1 $C $A $B
bash profiles/ab.sh r06ba 1 $B $C $A
bash profiles/ab.sh r06ba 1 $A $C $B
