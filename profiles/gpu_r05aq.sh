#!/bin/bash
# r05aq: A/B of the DPP wave scans (base) against the tree before them (prev) on one box
# timing-only builds without sigma's dW row (lbx1), its chain k-step (lbx2), its DMA (lbx3), all three (lbx4)
set -o pipefail
mkdir -p gpurun_out
for v in base prev base prev; do
  lib=deblur-e-nerf_amd/libden.so; [ $v != base ] && lib=deblur-e-nerf_amd/libden_$v.so
  DEN_LIB=$lib timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --psnr-steps 0 --no-extra-legs > gpurun_out/r05aq_$v.json 2> gpurun_out/r05aq_$v.err || exit $?
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r05aq_$v.json').read().splitlines()[-1]); k=d['roofline']['kernels']
print('$v', d['ms_per_step'], {n: v['avg_ms'] for n, v in k.items()})" | tee -a gpurun_out/r05aq_summary.txt
done
