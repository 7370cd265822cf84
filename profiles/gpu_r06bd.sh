# Round 6, call BD: folded L1 tuning -- v1: no S' in-flight fence in its dW phase; v2: v1 + a 9th W^T
# k-step in LDS and dz read two k-steps ahead -- fold parity test on each, then the A/B in all positions
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
for v in v1 v2; do
  DEN_LIB=$D/libden_$v.so timeout -k 10 300 python -u -m pytest tests/test_pe_fold_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06bd_pytest_$v.log 2>&1
  tail -1 gpurun_out/r06bd_pytest_$v.log
done
A=$D/libden.so; B=$D/libden_v1.so; C=$D/libden_v2.so
bash profiles/ab.sh r06bd 1 $A $B $C
bash profiles/ab.sh r06bd 1 $C $A $B
bash profiles/ab.sh r06bd 1 $B $C $A
bash profiles/ab.sh r06bd 1 $A $C $B
