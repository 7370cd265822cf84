# wave-per-event pixel-bandwidth forward (base) vs one thread per event (pf0)
# parity (pixel-bandwidth tests + the training-step tests), then the configs[3] emulation and the
# configs[2] bench line
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pixbw_gpu.py tests/test_deblur_gpu.py tests/test_train_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/tpixf.log 2>&1 || echo PARITY_FAIL >> gpurun_out/pixf.txt
for v in base pf0 base pf0; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/pixf.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/pixf.txt
  DEN_LIB=$lib timeout -k 10 200 python bench.py --pixbw --steps 10 --warmup 3 2>/dev/null | grep '^{' >> gpurun_out/pixf.txt
done
