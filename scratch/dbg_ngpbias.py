"""Debug: per-element error of the ngp base hidden-layer bias gradient (step_ngp_nopixbw_rd1)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "deblur-e-nerf_amd")]
import numpy as np, torch
import test_deblur_gpu as T
from test_nerfacc_gpu import _Draws
from deblur_e_nerf.external import marching
z = np.load(os.path.join(ROOT, "tests/golden/step_ngp_nopixbw_rd1.npz"))
m = T.build_model(z); m.train()
jit = [z[f"jitter_{i}"] for i in range(4)]
marching._uniform = _Draws([z["occ_u"], np.concatenate(jit)])
loss = m.training_step(T._batch(z), 0)
loss.backward(); torch.cuda.synchronize()
np.set_printoptions(linewidth=200, precision=3)
for k, p in m.nerf.radiance_field.named_parameters():
    if "params" in k:
        continue
    g = p.grad.detach().cpu().double().numpy().reshape(-1)
    r32, r64 = z[f"grad:{k}"].reshape(-1).astype(np.float64), z[f"grad:{k}_f64"].reshape(-1)
    e_our, e_ref = np.abs(g - r64), np.abs(r32 - r64)
    top = np.argsort(-e_our)[:6]
    print(f"{k}: |ours-f64| {np.linalg.norm(e_our):.3e} |ref32-f64| {np.linalg.norm(e_ref):.3e} |f64| {np.linalg.norm(r64):.3e}")
    for i in top:
        print(f"   [{i}] ours {g[i]:+.6e} ref32 {r32[i]:+.6e} f64 {r64[i]:+.6e}  err ours {e_our[i]:.2e} ref {e_ref[i]:.2e}")
