# Round 6, call BE: Lb two blocks ahead with 6 W^T k-steps in LDS, (lbe) plus the early derivative
# factors the registers now allow, (lbw) without them -- parity subset on lbe, A/B in all positions
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
DEN_LIB=$D/libden_lbe.so timeout -k 10 300 python -u -m pytest tests/test_pe_fold_gpu.py tests/test_train_gpu.py tests/test_render_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06be_pytest.log 2>&1
tail -1 gpurun_out/r06be_pytest.log
A=$D/libden.so; B=$D/libden_lbe.so; C=$D/libden_lbw.so
bash profiles/ab.sh r06be 1 $A $B $C
bash profiles/ab.sh r06be 1 $C $A $B
bash profiles/ab.sh r06be 1 $B $C $A
bash profiles/ab.sh r06be 1 $A $C $B
