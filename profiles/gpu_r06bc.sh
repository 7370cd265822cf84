# Round 6, call BC: phase split of the folded L1 launch (PEM 2) and Lb, DEN_HIDDEN_PROF build
set -e
set -o pipefail
mkdir -p gpurun_out
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_hidprof.so timeout -k 10 200 python -u profiles/hidden_prof.py 20 > gpurun_out/r06bc_hidden_prof.json 2> gpurun_out/r06bc_hidden_prof.err
cat gpurun_out/r06bc_hidden_prof.json
