# A/B of the pixel-bandwidth-on bench line (configs[2]) between libden builds
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  DEN_LIB=$lib timeout -k 10 240 python bench.py --pixbw --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/pixab_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/pixab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], {k: v['step_ms'] for k, v in d['roofline']['kernels'].items()})"
done
