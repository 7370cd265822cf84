"""Parity of the HIP render path (libden.so) against the oracle and the
reference's own golden vectors.  Needs an MI355X (marked gpu).

Tolerances (north_star: 1e-4 relative fp32):
* F32 parity mode: outputs |a-b| <= 1e-4 * max(|b|, 1); gradients 1e-4 tensor-wise
  relative (||a-b||/||b||).
* BF16 perf mode: bf16 operands (8-bit mantissa) through 11 layers -- checked
  against the same oracle with a looser bound stated per test.
"""
import os

import numpy as np
import pytest
import torch

from _util import flat_from_params, norm_rel, rel_err, synthetic_rays, unflat
from oracle import nerf as onerf

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _nat():
    from deblur_e_nerf import _native
    return _native


def _cfg(mode, rd, near=1.43, far=6.63):
    return dict(mode=_nat().mode_id(mode), rd=rd, aabb=list(onerf.AABB_CHAIR), near=near, far=far)


# ----------------------------------------------------------------------------- radiance field vs reference
@pytest.mark.parametrize("rd", [3, 1])
@pytest.mark.parametrize("mode,tol_out,tol_grad", [("f32", 1e-4, 1e-4), ("bf16", 3e-2, 5e-2)])
def test_field_matches_reference_golden(golden_dir, rd, mode, tol_out, tol_grad):
    nat = _nat()
    z = np.load(os.path.join(golden_dir, f"mlp_rd{rd}.npz"))
    p = onerf.build_params(rd, int(z["seed"]))
    flat = flat_from_params(p, rd).to(DEV).requires_grad_(True)
    packed = nat.PackedWeights(mode, rd, DEV)
    packed.pack(flat.detach())
    x = torch.from_numpy(z["x"]).to(DEV)
    d = torch.from_numpy(z["d"]).to(DEV)
    rgb, sig = nat.field(x, d, flat, _cfg(mode, rd), packed)
    e_rgb = rel_err(rgb, z["rgb_f32"])
    e_sig = rel_err(sig, z["sigma_f32"][:, 0])
    print(f"[{mode} rd={rd}] field rgb err {e_rgb:.2e} sigma err {e_sig:.2e}")
    assert e_rgb <= tol_out and e_sig <= tol_out
    loss = (rgb * torch.from_numpy(z["g_rgb"]).to(DEV)).sum() + (sig * torch.from_numpy(z["g_sigma"][:, 0]).to(DEV)).sum()
    loss.backward()
    g = unflat(flat.grad.detach().cpu(), rd)
    worst = 0.0
    for name in z["param_names"]:
        name = str(name)
        if f"grad:{name}" in z.files:
            e = norm_rel(g[name], z[f"grad:{name}"])
        else:
            ref_norm = float(z[f"gnorm_f32:{name}"])
            e = abs(float(g[name].double().norm()) - ref_norm) / max(ref_norm, 1e-30)
        if mode == "bf16" and g[name].numel() < 8:
            # a few scalar biases are sums of ~500 cancelling bf16 terms (the rgb bias
            # of rd=1 is 0.086 from terms of total magnitude ~200): bound their error
            # layer-relatively, by the reference gradient of the same layer's weight
            wname = name.replace(".bias", ".weight")
            ref = torch.from_numpy(z[f"grad:{name}"]).double()
            wref = torch.from_numpy(z[f"grad:{wname}"]).double()
            e = float((g[name].double() - ref).norm() / wref.norm())
        worst = max(worst, e)
        assert e <= tol_grad, (name, e)
    print(f"[{mode} rd={rd}] worst grad err {worst:.2e}")


# ----------------------------------------------------------------------------- full render vs oracle
@pytest.mark.parametrize("mode,n_samples,rd,bk", [("f32", 128, 3, True), ("f32", 64, 1, False),
                                                  ("bf16", 128, 3, True), ("bf16", 64, 1, True)])
def test_render_matches_oracle(mode, n_samples, rd, bk):
    nat = _nat()
    tol_out, tol_grad = (1e-4, 1e-4) if mode == "f32" else (3e-2, 6e-2)
    R = 16 if n_samples == 128 else 24
    o, d, u = synthetic_rays(R, seed=7 + rd)
    # a ray that misses the box and a ray starting inside it
    o[0] = torch.tensor([0.0, 5.0, -4.0]); d[0] = torch.tensor([0.0, 0.0, 1.0])
    o[1] = torch.tensor([0.2, -0.1, 0.3])
    p = onerf.build_params(rd, 3)
    for k in p:
        p[k].requires_grad_(True)
    bkgd = torch.tensor([0.9, 0.8, 0.7][:rd], requires_grad=True) if bk else None
    col, op, dep, _ = onerf.render_rays(p, o, d, u, n_samples=n_samples, bkgd=bkgd)
    g = torch.Generator().manual_seed(5)
    gc, go, gd = torch.randn(col.shape, generator=g), torch.randn(op.shape, generator=g), torch.randn(dep.shape, generator=g)
    ((col * gc).sum() + (op * go).sum() + (dep * gd).sum()).backward()

    flat = flat_from_params({k: v.detach() for k, v in p.items()}, rd).to(DEV).requires_grad_(True)
    packed = nat.PackedWeights(mode, rd, DEV)
    packed.pack(flat.detach())
    bk_dev = bkgd.detach().to(DEV).requires_grad_(True) if bk else None
    c2, o2, d2 = nat.render(o.to(DEV), d.to(DEV), u.to(DEV), bk_dev, flat, _cfg(mode, rd), packed, n_samples)
    d2n = d2 / (o2 + 1e-10)
    errs = (rel_err(c2, col), rel_err(o2, op), rel_err(d2n, dep))
    print(f"[{mode} S={n_samples} rd={rd}] colour/opacity/depth err {errs}")
    assert max(errs) <= tol_out * (1 if mode == "f32" else 4)
    ((c2 * gc.to(DEV)).sum() + (o2 * go.to(DEV)).sum() + (d2n * gd.to(DEV)).sum()).backward()
    gflat = unflat(flat.grad.cpu(), rd)
    worst = 0.0
    for k, v in p.items():
        e = norm_rel(gflat[k], v.grad)
        worst = max(worst, e)
        assert e <= tol_grad, (k, e)
    if bk:
        assert norm_rel(bk_dev.grad.cpu(), bkgd.grad) <= tol_grad
    print(f"[{mode} S={n_samples} rd={rd}] worst grad err {worst:.2e}")


def test_render_rejects_bad_shapes():
    nat = _nat()
    flat = torch.zeros(nat.param_count(3), device=DEV)
    packed = nat.PackedWeights("bf16", 3, DEV)
    packed.pack(flat)
    o, d, u = synthetic_rays(3, device=DEV)
    with pytest.raises(nat.DenError):
        nat.render(o, d, u, None, flat, _cfg("bf16", 3), packed, 128)  # 3 rays x 128 is not a tile multiple
