# Round 6, call BG: only waves 0..3 issue the ring DMA (the second wave per SIMD freed of it) -- judged on
# Lb (spill-free; the plain L variant spills 4 in this build): parity subset, then ABBA
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
DEN_LIB=$D/libden_ndw4.so timeout -k 10 300 python -u -m pytest tests/test_pe_fold_gpu.py tests/test_train_gpu.py tests/test_render_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06bg_pytest.log 2>&1
tail -1 gpurun_out/r06bg_pytest.log
A=$D/libden.so; B=$D/libden_ndw4.so
bash profiles/ab.sh r06bg 1 $A $B
bash profiles/ab.sh r06bg 1 $B $A
bash profiles/ab.sh r06bg 1 $A $B
bash profiles/ab.sh r06bg 1 $B $A
