#!/bin/bash
# r05be: forward compositing split over four waves on the four SIMDs at three gaps (base) vs one wave per ray at one gap (prev):
# GPU suite, forward cycle split, then A/B on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r05be_tests.log 2>&1 || exit $?
DEN_LIB=deblur-e-nerf_amd/libden_fprof.so timeout -k 10 240 python -u profiles/fwd_prof.py train > gpurun_out/r05be_fwd_prof.txt 2>&1 || exit $?
for v in base prev base prev base prev; do
  lib=deblur-e-nerf_amd/libden.so; [ $v != base ] && lib=deblur-e-nerf_amd/libden_$v.so
  DEN_LIB=$lib timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05be_$v.json 2> gpurun_out/r05be_$v.err || exit $?
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r05be_$v.json').read().splitlines()[-1]); k=d['roofline']['kernels']
print('$v', d['ms_per_step'], {n: v['avg_ms'] for n, v in k.items()})" | tee -a gpurun_out/r05be_summary.txt
done
