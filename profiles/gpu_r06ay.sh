# Round 6, call AY: the pe weight-gradient fold (L5 / L1 hidden launches, no streamed launch, dz_0 kept
# on chip): GPU suite on it, then ABBA A/B against the same tree built with -DDEN_NO_PE_FOLD
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ay_pytest.log 2>&1
tail -1 gpurun_out/r06ay_pytest.log
A=$D/libden_nofold.so; B=$D/libden.so
bash profiles/ab.sh r06ay 1 $A $B
bash profiles/ab.sh r06ay 1 $B $A
bash profiles/ab.sh r06ay 1 $A $B
bash profiles/ab.sh r06ay 1 $B $A
