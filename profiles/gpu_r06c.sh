# Round 6 (c): the hidden backward's phase split (DEN_HIDDEN_PROF build), L1 and Lb
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DEN_LIB=deblur-e-nerf_amd/libden_hidprof.so timeout -k 10 180 python -u profiles/hidden_prof.py 20 > gpurun_out/r06c_hidden_prof.json 2> gpurun_out/r06c_hidden_prof.err
DEN_LIB=deblur-e-nerf_amd/libden_hidprof.so timeout -k 10 180 python -u profiles/hidden_prof.py 20 >> gpurun_out/r06c_hidden_prof.json 2>> gpurun_out/r06c_hidden_prof.err
echo done
