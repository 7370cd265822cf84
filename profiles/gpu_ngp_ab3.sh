# ngp table-atomic pre-aggregation: parity of the variants, then ngp_bench + configs[3] emulation A/B
set -e
mkdir -p gpurun_out
for v in agg128 aggall; do
  DEN_LIB=deblur-e-nerf_amd/libden_$v.so timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_$v.log 2>&1
done
for v in base agg128 aggall base agg128 aggall; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/ngp_ab3.txt
  DEN_LIB=$lib timeout -k 10 120 python profiles/ngp_bench.py 2>/dev/null | grep '^{' >> gpurun_out/ngp_ab3.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/ngp_ab3.txt
done
