# ngp MFMA kernels templated on the hidden activation + fast softplus (base) vs libm softplus
# (slowact) vs the runtime activation switch (notmpl); parity, ngp_bench / configs[3] A/B, then the
# memory-side atomic request count of the backward (TCC_EA0_ATOMIC)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ngp_gpu.py tests/test_deblur_gpu.py -k "ngp" -q --timeout 120 --timeout-method thread > gpurun_out/tngp_act.log 2>&1 || echo PARITY_FAIL >> gpurun_out/ngp_act.txt
for v in base slowact notmpl base slowact notmpl; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  echo "== $v" >> gpurun_out/ngp_act.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/ngp_bench.py 2>/dev/null | grep '^{' >> gpurun_out/ngp_act.txt
  DEN_LIB=$lib timeout -k 10 200 python profiles/bench_ziggy.py --opt-steps 2 2>/dev/null | grep '^{' >> gpurun_out/ngp_act.txt
done
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_ATOMIC_sum --output-format csv -d gpurun_out/pmc_atom -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 0 --acc 2 > gpurun_out/pmc_atom.log 2>&1
