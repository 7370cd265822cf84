# per-wave cycle split of the persistent BF16 forward (DEN_FWD_PROF build)
set -e
mkdir -p gpurun_out
DEN_LIB=deblur-e-nerf_amd/libden_prof.so timeout -k 10 120 python profiles/fwd_prof.py train > gpurun_out/fprof.txt 2>&1
