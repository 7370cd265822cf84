DEN_LIB=deblur-e-nerf_amd/libden_prof.so timeout -k 10 120 python profiles/fwd_prof.py train > gpurun_out/fprof.txt 2>&1
DEN_LIB=deblur-e-nerf_amd/libden_prof1.so timeout -k 10 120 python profiles/fwd_prof.py train >> gpurun_out/fprof.txt 2>&1
for t in nofix fix; do (cd _naniso/$t && timeout -k 10 300 python bench.py --pixbw --steps 6 --warmup 0 --no-cpu-baseline > ../../gpurun_out/nan_$t.log 2>&1) || break; done
timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -q -s --timeout 120 --timeout-method thread -k "bf16 or many_blocks or layer_major" > gpurun_out/t_bf16.log 2>&1
