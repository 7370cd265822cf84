"""Parity of the packed rendering path (nerfacc 0.3.1's marching / visibility / compositing /
occupancy grid, restated in den_march.hip) and of the trajectory kernel against fixtures the
REFERENCE's own code produced (tests/golden/make_golden.py: models/nerf.py NeRF.forward ->
external/utils.py render_image -> external/vol_rendering.py rendering, with nerfacc's
primitives restated by oracle/nerfacc.py; models/trajectories.py LinearTrajectory with RoMa
restated by oracle/roma.py).  Needs an MI355X (marked gpu).

Tolerances: marching samples bit-exact (the same sequential f32 arithmetic); compositing and
renders in F32 mode 1e-4 relative (north_star), gradients 1e-4 / 1e-3 tensor-wise relative;
trajectory positions 1e-6, rotations 2e-6 absolute (f32 transcendentals, ulp-level).
"""
import os

import numpy as np
import pytest
import torch

from _util import flat_from_params, norm_rel, rel_err
from oracle import nerf as onerf

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mods():
    from deblur_e_nerf import _native
    from deblur_e_nerf.external import marching
    from deblur_e_nerf.models import nerf as nerf_lib
    from deblur_e_nerf.utils.easydict import EasyDict
    return _native, marching, nerf_lib, EasyDict


ARCH = dict(net_depth=8, net_width=256, skip_layer=4, net_depth_condition=1, net_width_condition=128,
            hidden_activation="softplus", density_activation="shifted_trunc_exp", radiance_activation="softplus",
            pos_encoder_max_deg=10, view_encoder_max_deg=4, weight_norm=False)


class _Draws:
    """Replays the U[0,1) draws a reference run recorded, in call order (marching._uniform)."""

    def __init__(self, arrays):
        self.arrays = list(arrays)

    def __call__(self, *size, device=None):
        a = torch.as_tensor(self.arrays.pop(0)).float()
        assert tuple(a.shape) == tuple(size), (a.shape, size)
        return a.to(device)


def build_nerf(z, mode="f32", sigma_shift=None):
    """Our NeRF in the fixture's configuration, weights = the reference's seeded init."""
    nat, marching, nerf_lib, ED = _mods()
    rd = int(z["rd"])
    occ = ED(resolution=int(z["res"]), occ_thre=0.01, ema_decay=0.95, warmup_steps=256, n=16)
    aabb = [float(v) for v in z["aabb"]]
    nerf = nerf_lib.NeRF(aabb, marching.ContractionType.AABB, occ, float(z["near"]), float(z["far"]),
                         float(z["step"]), "parameter", 0.0, 1e-4, 0.0, 16384, "mlp", ED(ARCH), 3, rd, mode=mode)
    p = onerf.build_params(rd, int(z["seed"]))
    nerf.radiance_field.flat_params.copy_(flat_from_params(p, rd))
    nerf = nerf.to(DEV)
    if sigma_shift is not None:
        with torch.no_grad():
            nerf.radiance_field.mlp.sigma_layer.output_layer.bias.add_(sigma_shift)
    return nerf


def _grad_pick(nerf):
    grads = [p.grad.detach().reshape(-1) for _, p in nerf.radiance_field.mlp.named_parameters()]
    return torch.cat(grads).cpu()


@pytest.mark.parametrize("rd", [1, 3])
def test_occupancy_grid_update_matches_reference(golden_dir, rd, monkeypatch):
    nat, marching, _, _ = _mods()
    z = np.load(os.path.join(golden_dir, f"render_rd{rd}.npz"))
    nerf = build_nerf(z)
    nerf.train()
    monkeypatch.setattr(marching, "_uniform", _Draws([z["occ_u"]]))
    nerf.update_occ_grid(step=0, T_wc_position=torch.from_numpy(z["rays_o"]).to(DEV))
    occs = nerf.occupancy_grid.occs.cpu()
    e = rel_err(occs, z["occs"])
    binary = nerf.occupancy_grid.binary.cpu().numpy()
    flips = int((binary != z["binary"]).sum())
    print(f"[rd={rd}] occs err {e:.2e}, binary flips {flips} of {binary.size}, occupied {binary.mean():.3f}")
    assert e <= 1e-4
    # a cell flips only if its occupancy sits at the mean threshold within the f32 noise
    thr = min(float(z["occs"].mean()), 0.01)
    near = np.abs(z["occs"].reshape(binary.shape) - thr) <= 1e-4 * thr
    assert ((binary != z["binary"]) & ~near).sum() == 0


@pytest.mark.parametrize("rd", [1, 3])
def test_marching_matches_reference_samples(golden_dir, rd):
    """den_march_prep/count/fill against the reference run's packed samples (before and after
    the early-stop pre-pass is applied: the marched set is bit-exact)."""
    nat, marching, _, _ = _mods()
    z = np.load(os.path.join(golden_dir, f"render_rd{rd}.npz"))
    import ctypes
    o = torch.from_numpy(z["rays_o"]).to(DEV)
    d = torch.from_numpy(z["rays_d"]).to(DEV)
    R = o.shape[0]
    L = nat.lib()
    tmin = torch.empty(R, device=DEV)
    tmax = torch.empty(R, device=DEV)
    jit = torch.from_numpy(z["train_jitter"]).float().to(DEV)
    ab = marching._carr(ctypes.c_float, [float(v) for v in z["aabb"]])
    nat._check(L.den_march_prep(R, nat._ptr(o), nat._ptr(d), ab, float(z["near"]), float(z["far"]), nat._ptr(jit),
                                float(z["step"]), nat._ptr(tmin), nat._ptr(tmax), nat._stream()))
    assert torch.equal(tmin.cpu(), torch.from_numpy(z["train_t_min"]))
    assert torch.equal(tmax.cpu(), torch.from_numpy(z["train_t_max"]))
    grid = marching.OccupancyGrid([float(v) for v in z["aabb"]], int(z["res"])).to(DEV)
    grid._binary.copy_(torch.from_numpy(z["binary_render"]))
    roi, res, binary, ct = marching._grid_args(grid)
    counts = torch.empty(R, dtype=torch.int32, device=DEV)
    args = (R, nat._ptr(o), nat._ptr(d), nat._ptr(tmin), nat._ptr(tmax), roi, res, nat._ptr(binary), ct,
            float(z["step"]), 0.0)
    nat._check(L.den_march_count(*args, nat._ptr(counts), nat._stream()))
    off, n = marching._scan(counts)
    ri = torch.empty(n, dtype=torch.int32, device=DEV)
    t0 = torch.empty(n, device=DEV)
    t1 = torch.empty(n, device=DEV)
    nat._check(L.den_march_fill(*args, nat._ptr(off), nat._ptr(ri), nat._ptr(t0), nat._ptr(t1), nat._stream()))
    print(f"[rd={rd}] marched {n} samples (reference {len(z['train_marched_ri'])})")
    assert n == len(z["train_marched_ri"])
    assert np.array_equal(ri.cpu().numpy(), z["train_marched_ri"])
    assert np.array_equal(t0.cpu().numpy(), z["train_marched_t0"])
    assert np.array_equal(t1.cpu().numpy(), z["train_marched_t1"])


@pytest.mark.parametrize("ctype,cone", [(2, 0.004), (1, 0.004), (2, 0.0)])
def test_marching_unbounded_matches_oracle(ctype, cone):
    """The wave-parallel march (den_march_count / fill for the sphere and tanh contractions: every
    lane runs the step chain, lanes test 64 steps at once) against oracle/nerfacc.march's sequential
    loop: bit-exact samples, including a ray that misses (near > far) and configs[3]'s near 0.01,
    far 13, cone angle 0.004 on a random 32^3 grid."""
    import ctypes
    from oracle import nerfacc as onacc
    nat, marching, _, _ = _mods()
    g = torch.Generator().manual_seed(5 + ctype)
    R = 24
    aabb = [0.2, -0.4, 0.0, 3.7, 3.7, 1.8]
    lo, hi = torch.tensor(aabb[:3]), torch.tensor(aabb[3:])
    o = lo + torch.rand(R, 3, generator=g) * (hi - lo)
    d = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1)
    tmin = torch.full((R,), 0.01) + torch.rand(R, generator=g) * 0.005
    tmax = torch.full((R,), 13.0)
    tmin[3], tmax[3] = 1e10, 1e10  # a miss
    res = [32, 32, 32]
    binary = (torch.rand(*res, generator=g) < 0.3).to(torch.uint8)
    step = 0.005
    ri_r, t0_r, t1_r, cnt_r = onacc.march(o.numpy(), d.numpy(), tmin.numpy(), tmax.numpy(), binary.numpy(),
                                          np.asarray(aabb, np.float32), res, ctype, step, cone)
    L = nat.lib()
    od, dd, tmin_d, tmax_d, bin_d = (t.to(DEV) for t in (o, d, tmin, tmax, binary))
    args = (R, nat._ptr(od), nat._ptr(dd), nat._ptr(tmin_d), nat._ptr(tmax_d), marching._carr(ctypes.c_float, aabb),
            marching._carr(ctypes.c_int32, res), nat._ptr(bin_d), ctype, step, cone)
    counts = torch.empty(R, dtype=torch.int32, device=DEV)
    nat._check(L.den_march_count(*args, nat._ptr(counts), nat._stream()))
    off, n = marching._scan(counts)
    ri = torch.empty(n, dtype=torch.int32, device=DEV)
    t0 = torch.empty(n, device=DEV)
    t1 = torch.empty(n, device=DEV)
    nat._check(L.den_march_fill(*args, nat._ptr(off), nat._ptr(ri), nat._ptr(t0), nat._ptr(t1), nat._stream()))
    print(f"[ctype={ctype} cone={cone}] {n} samples (oracle {len(ri_r)}), max per ray {int(cnt_r.max())}")
    assert np.array_equal(counts.cpu().numpy(), cnt_r) and cnt_r[3] == 0 and n > 0
    assert np.array_equal(ri.cpu().numpy(), ri_r)
    assert np.array_equal(t0.cpu().numpy(), t0_r) and np.array_equal(t1.cpu().numpy(), t1_r)


@pytest.mark.parametrize("rd", [1, 3])
def test_vol_rendering_matches_reference(golden_dir, rd):
    """external/vol_rendering.rendering on explicit packed samples: colours / opacities / depths
    and the gradients to sigma, rgb and the background."""
    nat, marching, _, _ = _mods()
    z = np.load(os.path.join(golden_dir, f"render_rd{rd}.npz"))
    T = lambda k: torch.from_numpy(z[k]).to(DEV)  # noqa: E731
    sig = T("vr_sigma").requires_grad_(True)
    rgb = T("vr_rgb").requires_grad_(True)
    bk = T("vr_bkgd").requires_grad_(True)
    from deblur_e_nerf.external.vol_rendering import rendering
    col, op, dp = rendering(T("vr_t0"), T("vr_t1"), T("vr_ri"), 24, rgb_sigma_fn=lambda a, b, c: (rgb, sig),
                            render_bkgd=bk)
    for a, k in ((col, "vr_color"), (op, "vr_opacity"), (dp, "vr_depth")):
        e = rel_err(a, z[k])
        assert e <= 1e-5, (k, e)
    ((col * T("vr_gc")).sum() + (op * T("vr_go")).sum() + (dp * T("vr_gd")).sum()).backward()
    for a, k in ((sig.grad, "vr_dsigma"), (rgb.grad, "vr_drgb"), (bk.grad, "vr_dbkgd")):
        e = norm_rel(a, z[k])
        print(f"[rd={rd}] {k} err {e:.2e}")
        assert e <= 1e-5, (k, e)


@pytest.mark.parametrize("rd", [1, 3])
def test_vol_rendering_alpha_matches_density(golden_dir, rd):
    """rendering(rgb_alpha_fn=...) (nerfacc render_weight_from_alpha, vol_rendering.py:96-106) on
    alpha_i = 1 - exp(-sigma_i (t1 - t0)) renders what rgb_sigma_fn renders from sigma_i, and its
    alpha gradient maps to the sigma gradient by the chain rule (d alpha / d sigma = dt exp(-sigma dt))."""
    from deblur_e_nerf.external.vol_rendering import rendering
    z = np.load(os.path.join(golden_dir, f"render_rd{rd}.npz"))
    T = lambda k: torch.from_numpy(z[k]).to(DEV)  # noqa: E731
    t0, t1 = T("vr_t0"), T("vr_t1")
    sig = T("vr_sigma").requires_grad_(True)
    rgb = T("vr_rgb")
    dt = (t1 - t0).reshape(sig.shape)
    alpha = (1 - torch.exp(-sig.detach() * dt)).requires_grad_(True)
    grads = (T("vr_gc"), T("vr_go"), T("vr_gd"))
    outs_s = rendering(t0, t1, T("vr_ri"), 24, rgb_sigma_fn=lambda a, b, c: (rgb, sig), render_bkgd=T("vr_bkgd"))
    outs_a = rendering(t0, t1, T("vr_ri"), 24, rgb_alpha_fn=lambda a, b, c: (rgb, alpha), render_bkgd=T("vr_bkgd"))
    for a, b in zip(outs_a, outs_s):
        assert rel_err(a.detach(), b.detach().cpu().numpy()) <= 1e-5
    sum((o * g.reshape(o.shape)).sum() for o, g in zip(outs_s, grads)).backward()
    sum((o * g.reshape(o.shape)).sum() for o, g in zip(outs_a, grads)).backward()
    mapped = alpha.grad * dt * torch.exp(-sig.detach() * dt)
    assert norm_rel(mapped, sig.grad.detach().cpu().numpy()) <= 1e-4


@pytest.mark.parametrize("rd", [1, 3])
def test_nerf_forward_matches_reference(golden_dir, rd, monkeypatch):
    """NeRF.forward (sampler 'occupancy', F32): the reference's training-mode render with the
    recorded stratified jitter (samples after the early-stop pre-pass, radiance, opacity, depth,
    mean samples per ray), its backward (MLP and background gradients), and the eval render."""
    nat, marching, _, _ = _mods()
    z = np.load(os.path.join(golden_dir, f"render_rd{rd}.npz"))
    nerf = build_nerf(z, sigma_shift=float(z["sigma_bias_shift"]))
    nerf.occupancy_grid._binary.copy_(torch.from_numpy(z["binary_render"]).to(DEV))
    nerf.train()
    o = torch.from_numpy(z["rays_o"]).to(DEV)
    d = torch.from_numpy(z["rays_d"]).to(DEV)
    monkeypatch.setattr(marching, "_uniform", _Draws([z["train_jitter"]]))
    rad, op, dp, mspr = nerf(o, d)
    print(f"[rd={rd}] mean samples/ray {mspr:.3f} (reference {float(z['train_mspr']):.3f})")
    assert abs(mspr - float(z["train_mspr"])) <= 2.0 / o.shape[0]
    for a, k in ((rad, "train_radiance"), (op, "train_opacity"), (dp, "train_depth")):
        e = rel_err(a, z[k])
        print(f"[rd={rd}] {k} err {e:.2e}")
        assert e <= 1e-4, (k, e)
    g = lambda k: torch.from_numpy(z[k]).to(DEV)  # noqa: E731
    ((rad * g("g_rad")).sum() + (op * g("g_op")).sum() + (dp * g("g_dp")).sum()).backward()
    flat = _grad_pick(nerf)
    idx = torch.from_numpy(z["grad_pick_idx"])
    e_pick = norm_rel(flat[idx], z["grad_pick"])
    e_norm = abs(float(flat.double().norm()) - float(z["grad_norm"])) / float(z["grad_norm"])
    e_bk = norm_rel(nerf.parametrizations.render_bkgd.original.grad, z["grad_bkgd_orig"])
    print(f"[rd={rd}] grad pick err {e_pick:.2e}, norm err {e_norm:.2e}, bkgd err {e_bk:.2e}")
    assert e_pick <= 1e-3 and e_norm <= 1e-4 and e_bk <= 1e-4
    for k, p in nerf.radiance_field.mlp.named_parameters():
        if f"grad:{k}" in z.files:
            e = norm_rel(p.grad.reshape(-1), z[f"grad:{k}"])
            assert e <= 1e-3, (k, e)
    nerf.eval()
    with torch.no_grad():
        rad, op, dp, mspr = nerf(o, d)
    for a, k in ((rad, "eval_radiance"), (op, "eval_opacity"), (dp, "eval_depth")):
        assert rel_err(a, z[k]) <= 1e-4, k
    assert abs(mspr - float(z["eval_mspr"])) <= 2.0 / o.shape[0]


def test_trajectory_matches_reference(golden_dir):
    nat = _mods()[0]
    z = np.load(os.path.join(golden_dir, "traj.npz"))
    from deblur_e_nerf.data.datasets import CameraPose
    from deblur_e_nerf.models.trajectories import LinearTrajectory
    cp = CameraPose.from_arrays(z["T_wc_position"], z["T_wc_orientation"], z["T_wc_timestamp"])
    traj = LinearTrajectory(cp).to(DEV)
    for q, pk, rk in (("query_ts", "position", "rotation"), ("query_ts_2d", "position_2d", "rotation_2d")):
        p, r = traj(torch.from_numpy(z[q]).to(DEV))
        ep = float((p.cpu() - torch.from_numpy(z[pk])).abs().max())
        er = float((r.cpu() - torch.from_numpy(z[rk])).abs().max())
        print(f"trajectory {q}: position err {ep:.2e}, rotation err {er:.2e}")
        assert p.shape == z[pk].shape and ep <= 1e-6 and er <= 2e-6
    traj.check()
    traj(torch.tensor([float(z["T_wc_timestamp"][-1]) + 1.0], dtype=torch.float64, device=DEV))
    with pytest.raises(AssertionError):
        traj.check()


def test_vol_rendering_alpha_saturated_matches_autograd():
    """rgb_alpha_fn with alphas at and beyond 1 (the kernel's min(alpha, 1)): renders and the alpha /
    rgb / background gradients against torch autograd of the product form in f64 on the CPU
    (w_i = a_i prod_{j<i} (1 - a_j), a = clamp(alpha, max=1)).  Ragged rays across the 64-sample
    wave blocks, an empty ray, alpha = 0, alpha = 1 mid-ray (its derivative keeps the later samples'
    terms) and alpha > 1 (zero derivative)."""
    from deblur_e_nerf.external.vol_rendering import rendering
    gen = torch.Generator().manual_seed(11)
    lens = [0, 1, 5, 63, 64, 65, 130, 200, 17, 90]
    R, rd = len(lens), 3
    ri = torch.cat([torch.full((n,), r, dtype=torch.int32) for r, n in enumerate(lens)])
    n = ri.numel()
    t0 = torch.rand(n, 1, generator=gen)
    t1 = t0 + torch.rand(n, 1, generator=gen) * 0.1
    alpha = torch.rand(n, 1, generator=gen) * 0.08
    starts = torch.tensor([0] + lens).cumsum(0)
    alpha[starts[2] + 2] = 1.0     # saturates ray 2 mid-way
    alpha[starts[6] + 70] = 1.0    # ray 6, second wave block
    alpha[starts[7] + 10] = 1.3    # ray 7: clamp active, zero derivative
    alpha[starts[8] + 3] = 0.0
    rgb = torch.rand(n, rd, generator=gen)
    bk = torch.rand(rd, generator=gen)
    gc, go, gd = torch.randn(R, rd, generator=gen), torch.randn(R, 1, generator=gen), torch.randn(R, 1, generator=gen)

    a_d, rgb_d, bk_d = (v.double().requires_grad_(True) for v in (alpha, rgb, bk))
    cols, ops, dps = [], [], []
    for r in range(R):
        sl = slice(int(starts[r]), int(starts[r + 1]))
        a = a_d[sl, 0].clamp(max=1.0)
        T = torch.cat([torch.ones(1, dtype=torch.float64), torch.cumprod(1 - a, 0)[:-1]])
        w = a * T
        op = w.sum()
        cols.append((w[:, None] * rgb_d[sl]).sum(0) + bk_d * (1 - op))
        ops.append(op.reshape(1))
        dps.append((w * ((t0[sl, 0] + t1[sl, 0]).double() / 2)).sum().reshape(1))
    col_r, op_r, dp_r = torch.stack(cols), torch.stack(ops), torch.stack(dps)
    ((col_r * gc.double()).sum() + (op_r * go.double()).sum() + (dp_r * gd.double()).sum()).backward()

    a_g, rgb_g, bk_g = (v.to(DEV).requires_grad_(True) for v in (alpha, rgb, bk))
    col, op, dp = rendering(t0.to(DEV), t1.to(DEV), ri.to(DEV), R, rgb_alpha_fn=lambda a, b, c: (rgb_g, a_g),
                            render_bkgd=bk_g)
    for x, ref in ((col, col_r), (op, op_r), (dp, dp_r)):
        assert float((x.detach().cpu().double() - ref.detach()).abs().max()) <= 2e-6
    ((col * gc.to(DEV)).sum() + (op * go.to(DEV)).sum() + (dp * gd.to(DEV)).sum()).backward()
    for x, ref, k in ((a_g.grad, a_d.grad, "alpha"), (rgb_g.grad, rgb_d.grad, "rgb"), (bk_g.grad, bk_d.grad, "bkgd")):
        e = float((x.cpu().double() - ref).abs().max() / ref.abs().max())
        print(f"  d{k}: max err {e:.2e}")
        assert e <= 1e-5, k
    assert float(a_g.grad[starts[7] + 10]) == 0.0
    assert float(a_d.grad[starts[2] + 2].abs()) > 0 and float(a_g.grad[starts[2] + 2].abs()) > 0
