"""Debug: which samples of a points-mode / fixed-sampler render come out non-finite or wrong
(persistent forward bring-up)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "deblur-e-nerf_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from _util import flat_from_params, synthetic_rays  # noqa: E402
from oracle import nerf as onerf  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402

for mode in ("f32", "bf16"):
    rd, S = 3, 128
    R = 8 * nat.wg_samples(mode) // S * 37  # 37 items of the forward
    o, d, u = synthetic_rays(R, seed=11)
    p = onerf.build_params(rd, 0)
    flat = flat_from_params(p, rd).cuda()
    packed = nat.PackedWeights(mode, rd, "cuda")
    packed.pack(flat)
    cfg = dict(mode=nat.mode_id(mode), rd=rd, aabb=list(onerf.AABB_CHAIR), near=1.43, far=6.63)
    with torch.no_grad():
        c, op, _ = nat.render(o.cuda(), d.cuda(), u.cuda(), torch.ones(rd, device="cuda"), flat, cfg, packed, S)
    torch.cuda.synchronize()
    ref, ref_o, _, _ = onerf.render_rays(p, o, d, u, n_samples=S, bkgd=torch.ones(rd))
    c = c.cpu()
    bad = ~torch.isfinite(c).all(1)
    err = (c - ref).abs().max(1).values
    per = nat.wg_samples(mode) // S * (8 if mode == "bf16" else 8)
    print(mode, "rays", R, "nonfinite", int(bad.sum()), "first bad rays", bad.nonzero()[:10, 0].tolist(),
          "max err", float(err[~bad].max()) if (~bad).any() else None)
    print("  err per item (first 12):", [round(float(err[i * (256 // S):(i + 1) * (256 // S)].max()), 6)
                                         for i in range(12)])
