# ngp fold depth: parity (default quads and the deepest fold), then the configs[3] emulation A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_base.log 2>&1
DEN_LIB=deblur-e-nerf_amd/libden_s5.so timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_s5.log 2>&1
for v in base s3 s4 s5 base s3 s4 s5; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/ngp_ab4.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/ngp_ab4.txt
done
