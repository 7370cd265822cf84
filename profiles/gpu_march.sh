# wave-parallel marching for the unbounded contractions: parity (marching tests + the ngp / step
# tests that march), then the configs[3] emulation (base vs the per-thread march, libden_march1.so)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nerfacc_gpu.py tests/test_ngp_gpu.py tests/test_deblur_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/tmarch.log 2>&1 || echo PARITY_FAIL >> gpurun_out/march.txt
for v in base march1 base march1; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/march.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/march.txt
done
