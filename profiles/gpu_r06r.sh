# Round 6, call R: hidden phase split + clocks on the r06n tree, then Lb's sigma row inside the dW loop
# (rotated column order, DEN_HB_SIGMA_IN_DW) against the product, 3 alternating rounds.
set -e
set -o pipefail
mkdir -p gpurun_out
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_hidprof.so timeout -k 10 200 python -u profiles/hidden_prof.py > gpurun_out/r06r_hidden_prof.json 2> gpurun_out/r06r_hidden_prof.err
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_clock.so timeout -k 10 200 python -u profiles/clock_probe.py 4 r06r > gpurun_out/r06r_clock.jsonl 2> gpurun_out/r06r_clock.err
bash profiles/ab.sh r06r 3 $PWD/deblur-e-nerf_amd/libden.so $PWD/deblur-e-nerf_amd/libden_sigdw.so
