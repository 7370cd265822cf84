# Round 6, call BK: the whole library with -mllvm -amdgpu-mfma-vgpr-form (MFMA accumulators as arch VGPRs;
# spill-free): parity subset, then ABBA against the product
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
DEN_LIB=$D/libden_vgf.so timeout -k 10 300 python -u -m pytest tests/test_pe_fold_gpu.py tests/test_train_gpu.py tests/test_render_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06bk_pytest.log 2>&1
tail -1 gpurun_out/r06bk_pytest.log
A=$D/libden.so; B=$D/libden_vgf.so
bash profiles/ab.sh r06bk 1 $A $B
bash profiles/ab.sh r06bk 1 $B $A
bash profiles/ab.sh r06bk 1 $A $B
bash profiles/ab.sh r06bk 1 $B $A
