# Round 6, call AV: the hidden backward's phase split at 8 waves (L1 and Lb), DEN_HIDDEN_PROF build
set -e
set -o pipefail
mkdir -p gpurun_out
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_hidprof.so timeout -k 10 200 python -u profiles/hidden_prof.py 20 > gpurun_out/r06av_hidden_prof.json 2> gpurun_out/r06av_hidden_prof.err
cat gpurun_out/r06av_hidden_prof.json
