"""Debug: is the ngp density-bias gradient error in the field backward or upstream (compositing)?"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "deblur-e-nerf_amd")]
import numpy as np, torch
import test_deblur_gpu as T
from test_nerfacc_gpu import _Draws
from deblur_e_nerf.external import marching
from deblur_e_nerf import _native as nat
from oracle import ngp as ongp
z = np.load(os.path.join(ROOT, "tests/golden/step_ngp_nopixbw_rd1.npz"))
m = T.build_model(z); m.train()
cap = []
orig = nat.ngp_field_packed
def wrapped(flat, desc, rays_o, rays_d, ri, t0, t1, density_only=False):
    rgb, sig = orig(flat, desc, rays_o, rays_d, ri, t0, t1, density_only)
    if not density_only and rgb.requires_grad:
        rec = dict(o=rays_o.detach().cpu(), d=rays_d.detach().cpu(), ri=ri.detach().cpu(), t0=t0.detach().cpu(),
                   t1=t1.detach().cpu())
        rgb.register_hook(lambda g: rec.__setitem__("g_rgb", g.detach().cpu().clone()))
        sig.register_hook(lambda g: rec.__setitem__("g_sig", g.detach().cpu().clone()))
        cap.append(rec)
    return rgb, sig
nat.ngp_field_packed = wrapped
import deblur_e_nerf.external.ngp as ngpmod
ngpmod._native.ngp_field_packed = wrapped
jit = [z[f"jitter_{i}"] for i in range(4)]
marching._uniform = _Draws([z["occ_u"], np.concatenate(jit)])
loss = m.training_step(T._batch(z), 0)
loss.backward(); torch.cuda.synchronize()
rf = m.nerf.radiance_field
ours = {k: p.grad.detach().cpu().double() for k, p in rf.named_parameters()}
print("calls captured", len(cap), [len(c["ri"]) for c in cap])
# oracle field backward (f64) with OUR upstream gradients on OUR packed samples
p = {k: prm.detach().cpu().double().clone().requires_grad_(True) for k, prm in rf.named_parameters()}
pos = json.loads(str(z["pos_encoding"]))
aabb = torch.tensor([float(v) for v in z["aabb"]], dtype=torch.float64)
ctype = {"aabb": 0, "tanh": 1, "sphere": 2}[str(z["contraction"])]
for c in cap:
    ri = c["ri"].long()
    x = c["o"].double()[ri] + c["d"].double()[ri] * ((c["t0"].double() + c["t1"].double()) / 2.0).reshape(-1, 1)
    rgb, dens = ongp.field(p, x, c["d"].double()[ri], int(z["rd"]), aabb, ctype, pos)
    gr = c["g_rgb"].double().reshape(rgb.shape); gs = c["g_sig"].double().reshape(-1, 1)
    ((rgb * gr).sum() + (dens * gs).sum()).backward()
for k in ("mlp_base.1.output_layer.bias", "mlp_base.1.hidden_layers.0.bias", "mlp_base.1.output_layer.weight"):
    a, b = ours[k].reshape(-1), p[k].grad.reshape(-1)
    f64 = torch.from_numpy(z[f"grad:{k}_f64"]).double().reshape(-1)
    print(f"{k}: ours vs oracle-on-our-upstream {float((a - b).norm() / b.norm()):.3e}; oracle-on-our-upstream vs "
          f"reference f64 {float((b - f64).norm() / f64.norm()):.3e}")
    print("   [0..3] ours", a[:4].numpy(), "oracle", b[:4].numpy(), "f64", f64[:4].numpy())
