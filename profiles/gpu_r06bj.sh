# Round 6, call BJ: the whole library scheduled with -mllvm -amdgpu-sched-strategy=iterative-minreg
# (spill-free; forward at 220 VGPRs): parity subset, then ABBA against the product
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
DEN_LIB=$D/libden_iter.so timeout -k 10 300 python -u -m pytest tests/test_pe_fold_gpu.py tests/test_train_gpu.py tests/test_render_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06bj_pytest.log 2>&1
tail -1 gpurun_out/r06bj_pytest.log
A=$D/libden.so; B=$D/libden_iter.so
bash profiles/ab.sh r06bj 1 $A $B
bash profiles/ab.sh r06bj 1 $B $A
bash profiles/ab.sh r06bj 1 $A $B
bash profiles/ab.sh r06bj 1 $B $A
