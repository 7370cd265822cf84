# forward variants: NB (column blocks per wave) x explicit schedule pins; cycle split of the pinned NB=2 build
timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py tests/test_nerfacc_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_fwd.log 2>&1 || exit 1
DEN_LIB=deblur-e-nerf_amd/libden_prof.so timeout -k 10 120 python profiles/fwd_prof.py train > gpurun_out/fprof.txt 2>&1
bash profiles/exp_variants.sh fwd5 base nb2ns nb1s nb1ns base
