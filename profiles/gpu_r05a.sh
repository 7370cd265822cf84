#!/bin/bash
# r05a: GPU suite on the round-4 tree + PSNR-leg variance sweep (HIP F32, 4 batch sequences per variant)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05a_tests.log 2>&1 || exit $?
timeout -k 10 840 python -u profiles/psnr_sweep.py --seqs 4 --modes f32 --out gpurun_out/r05a_psnr_sweep.jsonl --variants '[
 {"n_events":128,"steps":3000,"milestones":[0.3,0.6,0.85],"teacher_rgb_scale":1.0},
 {"n_events":128,"steps":3000,"milestones":[0.3,0.6,0.85]},
 {"n_events":256,"steps":3000,"milestones":[0.3,0.6,0.85],"teacher_rgb_scale":1.0},
 {"n_events":128,"steps":3000,"milestones":[0.5,0.75,0.9],"lr_gamma":0.2,"teacher_rgb_scale":3.0,"n_views":8,"view":32},
 {"n_events":128,"steps":1500,"milestones":[0.3,0.6,0.85],"teacher_rgb_scale":1.0}
]' > gpurun_out/r05a_psnr.log 2>&1
