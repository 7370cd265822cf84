"""Shared test helpers (synthetic inputs, flat-parameter plumbing, tolerances)."""
import math

import numpy as np
import torch

from oracle import nerf as onerf


def synthetic_rays(R, seed=1234, radius=4.03, jitter_rad=0.3, device="cpu"):
    """camera centres on a sphere around the chair's AABB, rays
    towards the origin perturbed by up to +-0.3 rad; per-ray stratified jitter."""
    g = torch.Generator().manual_seed(seed)
    v = torch.randn(R, 3, generator=g)
    o = v / v.norm(dim=-1, keepdim=True) * radius
    d = -o / o.norm(dim=-1, keepdim=True) + (torch.rand(R, 3, generator=g) * 2 - 1) * math.sin(jitter_rad)
    d = d / d.norm(dim=-1, keepdim=True)
    u = torch.rand(R, generator=g)
    return o.to(device), d.to(device), u.to(device)


def flat_from_params(p, rd):
    names = [n for n, _, _ in onerf.layer_specs(rd)]
    return torch.cat([torch.cat([p[n + ".weight"].reshape(-1), p[n + ".bias"].reshape(-1)]) for n in names])


def unflat(flat, rd):
    out, off = {}, 0
    for n, fin, fout in onerf.layer_specs(rd):
        out[n + ".weight"] = flat[off:off + fin * fout].view(fout, fin)
        off += fin * fout
        out[n + ".bias"] = flat[off:off + fout]
        off += fout
    return out


def rel_err(a, b):
    a = np.asarray(torch.as_tensor(a).detach().cpu().double())
    b = np.asarray(torch.as_tensor(b).detach().cpu().double())
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0)))


def norm_rel(a, b):
    """||a - b|| / ||b|| (tensor-wise relative error, for gradients)."""
    a = torch.as_tensor(a).detach().cpu().double()
    b = torch.as_tensor(b).detach().cpu().double()
    return float((a - b).norm() / max(b.norm(), 1e-30))


# ----------------------------------------------------------------------------- ngp fixtures
NGP_CTYPE = {"aabb": 0, "tanh": 1, "sphere": 2}


def ngp_fixture(z):
    """(params {name: tensor}, pos_encoding cfg, base cfg, head cfg, rd, ctype) of a
    tests/golden/ngp_*.npz fixture; the default-size hash table is regenerated from the seed
    (oracle/ngp.build_params, x 1e3 as make_golden.gen_ngp) and checked against its stored sum."""
    import json
    from oracle import ngp as ongp
    pos = json.loads(str(z["pos_encoding"]))
    rd = int(z["rd"])
    if "table" in z.files:
        table = torch.from_numpy(z["table"])
    else:
        table = ongp.build_params(rd, int(z["seed"]), pos)["mlp_base.0.params"] * 1e3
        assert abs(table.double().sum().item() - float(z["table_sum"])) <= 1e-6 * max(1.0, abs(float(z["table_sum"])))
    p = {"mlp_base.0.params": table}
    for k in z.files:
        if k.startswith("param:"):
            p[k[len("param:"):]] = torch.from_numpy(z[k])
    base = dict(ongp.MLP_BASE, hidden_activation=str(z["hidden"]))
    head = dict(ongp.MLP_HEAD, hidden_activation=str(z["hidden"]), radiance_activation=str(z["radiance"]))
    return p, pos, base, head, rd, NGP_CTYPE[str(z["contraction"])]


def ngp_table_grad(z, n):
    """The fixture's hash-table gradient as a dense (n,) tensor."""
    if "grad:mlp_base.0.params" in z.files:
        return torch.from_numpy(z["grad:mlp_base.0.params"])
    g = torch.zeros(n)
    g[torch.from_numpy(z["table_grad_idx"]).long()] = torch.from_numpy(z["table_grad_val"])
    return g
