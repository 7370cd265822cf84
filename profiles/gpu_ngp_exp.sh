# experiment builds (wrong results, timing only): xnoat = backward without the table scatter,
# xlocal = forward gathers folded into the first 4096 entries (L2-resident); kernel traces of the
# configs[3] emulation for base / xnoat / xlocal
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base xnoat xlocal; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  DEN_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x_$v -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/x_$v.log 2>&1
done
