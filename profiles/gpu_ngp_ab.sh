# ngp A/B: parity tests of the new build, then ngp_bench + the configs[3] emulation, new vs old
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/tngp.log 2>&1
for v in base old base old; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/ngp_ab.txt
  DEN_LIB=$lib timeout -k 10 120 python profiles/ngp_bench.py 2>/dev/null | grep '^{' >> gpurun_out/ngp_ab.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/ngp_ab.txt
done
