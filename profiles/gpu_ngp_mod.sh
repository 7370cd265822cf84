# grid index without the runtime modulo where not needed (base) vs index % size always (mod0)
# Parity, then ngp_bench (2^19 random points) and the configs[3] emulation
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_mod.log 2>&1 || echo PARITY_FAIL >> gpurun_out/ngp_mod.txt
for v in base mod0 base mod0; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/ngp_mod.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/ngp_bench.py 2>/dev/null | grep '^{' >> gpurun_out/ngp_mod.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/ngp_mod.txt
done
