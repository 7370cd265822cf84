# dW kernel templated on the row-tile count (base) vs runtime shape (dw1)
# Parity, then ngp_bench (2^19 random points) and the configs[3] emulation
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_dwt.log 2>&1 || echo PARITY_FAIL >> gpurun_out/ngp_dwt.txt
for v in base dw1 base dw1; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/ngp_dwt.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/ngp_bench.py 2>/dev/null | grep '^{' >> gpurun_out/ngp_dwt.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/ngp_dwt.txt
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dwt_prof -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/dwt_prof.log 2>&1
