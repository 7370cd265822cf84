"""Debug: BF16 render gradients per layer at bench scale, hidden path of the loaded libden vs the
sample-major path (bwd_path=1), for A/B of backward variants."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "deblur-e-nerf_amd")]
import torch
import test_render_gpu as T
from _util import unflat, norm_rel

R = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
for rd in (3,):
    c1, g1, b1, _ = T._render_grads("bf16", rd, R, 128, seed=21)
    c2, g2, b2, _ = T._render_grads("bf16", rd, R, 128, seed=21, bwd_path=1)
    gf1, gf2 = unflat(g1.cpu(), rd), unflat(g2.cpu(), rd)
    for k in gf2:
        d = (gf1[k] - gf2[k]).abs()
        print(f"{k:40s} rel {norm_rel(gf1[k], gf2[k]):.2e} maxabs {float(d.max()):.2e} |g| {float(gf2[k].norm()):.3e}")
    print("bkgd", norm_rel(b1.cpu(), b2.cpu()), flush=True)
