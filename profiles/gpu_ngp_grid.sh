# field-kernel grid caps 512 / 768 / 1024 workgroups (4096 was the default): kernel traces of the configs[3] emulation
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in g512 g768 g1024; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  DEN_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/grid_$v -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 1 > gpurun_out/grid_$v.log 2>&1
done
