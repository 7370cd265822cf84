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
