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
    base = dict(ongp.MLP_BASE, hidden_activation=str(z["hidden"]),
                density_activation=str(z["density"]) if "density" in z.files else "shifted_trunc_exp")
    head = dict(ongp.MLP_HEAD, hidden_activation=str(z["hidden"]), radiance_activation=str(z["radiance"]))
    return p, pos, base, head, rd, NGP_CTYPE[str(z["contraction"])]


def ngp_table_grad(z, n):
    """The fixture's hash-table gradient as a dense (n,) tensor."""
    if "grad:mlp_base.0.params" in z.files:
        return torch.from_numpy(z["grad:mlp_base.0.params"])
    g = torch.zeros(n)
    g[torch.from_numpy(z["table_grad_idx"]).long()] = torch.from_numpy(z["table_grad_val"])
    return g


# the chair-like synthetic sequence of tests/golden/make_golden.py (EDS sensor constants)
EDS = dict(input_time_const_eff_it_prod=(35e-12 * 25e-3) / 2000e-12,
           miller_time_const_eff_it_prod=(0.6e-12 * 25e-3) / 2000e-12, amplifier_gain=140.0,
           closed_loop_gain=1 / 0.7, output_time_const=25e-6, sf_cutoff_freq=16400.0, diff_amp_cutoff_freq=82000.0)


def synthetic_dataset_arrays(rd=1, seed=61, C=64):
    """camera_calibration.npz + camera_poses.npz contents of a chair-like synthetic sequence:
    EDS-assumed sensor constants, contrast thresholds 0.25 / 0.2, refractory period 1 us, an
    800 x 800 f = 1111 camera circling the AABB at radius 4.03 (looking at the origin) over
    [0.05 s, 1.05 s]."""
    from scipy.spatial.transform import Rotation
    g = torch.Generator().manual_seed(seed)
    K = np.array([[1111.0, 0.0, 400.0], [0.0, 1111.0, 400.0], [0.0, 0.0, 1.0]], dtype=np.float32)
    cal = {k: np.array(v, dtype=np.float32) for k, v in EDS.items()}
    cal.update(pos_contrast_threshold=np.array(0.25, np.float32), neg_contrast_threshold=np.array(0.2, np.float32),
               refractory_period=np.array(1000, np.int64), intrinsics=K,
               bayer_pattern=np.array("RGGB" if rd == 3 else ""), img_height=np.array(800), img_width=np.array(800))
    ts = np.linspace(5e7, 1.05e9, C).astype(np.int64)
    ang = np.linspace(0.0, 1.2, C) + float(torch.rand(1, generator=g)) * 6.28
    pos = np.stack([4.03 * np.cos(ang), 4.03 * np.sin(ang), 0.6 + 0.2 * np.sin(3 * ang)], -1).astype(np.float32)
    rots = []
    for p in pos:
        z = -p / np.linalg.norm(p)
        x = np.cross(z, [0.0, 0.0, 1.0])
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        rots.append(np.stack([x, y, z], -1))
    quat = Rotation.from_matrix(np.stack(rots)).as_quat().astype(np.float32)  # XYZW
    poses = dict(T_wc_position=pos, T_wc_orientation=quat, T_wc_timestamp=ts)
    return cal, poses
