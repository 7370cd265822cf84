"""The render's gradient with respect to its RAYS and the chain behind it (render timestamps ->
LinearTrajectory -> NeRF.pixel_params_to_ray -> sample positions o + d t and view directions d):
den_render_ray_grad / den_ngp_ray_grad / den_pixel_rays_bwd / den_trajectory_bwd /
den_pixbw_sample_ts_bwd / den_pixbw_decay_ts_bwd against torch autograd of the oracle (the
reference's semantics: marching intervals detached, as nerfacc returns them).  This is the path of
the refractory period's gradient (deblur_e_nerf.py:419-455); tests/test_deblur_gpu.py checks the
whole chain against the reference training_step's dtau.  Needs an MI355X (marked gpu).

Tolerances: F32 parity mode, tensor-wise relative (||a - b|| / ||b||) against the f64 oracle, at
max(1e-4, 4 x the f32 oracle's own error) -- the high-frequency positional encoding (sin(2^9 x))
makes d/d(position) f32-conditioned at ~1e-4 in torch's f32 autograd as much as here; BF16 2e-2
(bf16 layer gradients, the field's own BF16 gradient bound is 3e-2).
"""
import numpy as np
import pytest
import torch

from _util import flat_from_params, norm_rel, synthetic_rays
from oracle import nerf as onerf

pytestmark = pytest.mark.gpu
DEV = "cuda"
CID = {"aabb": 0, "tanh": 1, "sphere": 2}


def _nat():
    from deblur_e_nerf import _native
    return _native


def _cfg(mode, rd, contraction="aabb", near=1.43, far=6.63):
    return dict(mode=_nat().mode_id(mode), rd=rd, aabb=list(onerf.AABB_CHAIR), near=near, far=far,
                contraction=CID[contraction])


def _floor(ref32, ref64, base=1e-4):
    """max(base, 4 x the f32 oracle's own tensor-wise error against f64)."""
    return max(base, 4.0 * norm_rel(ref32, ref64))


def _field_setup(mode, rd, seed):
    nat = _nat()
    p = onerf.build_params(rd, seed)
    flat = flat_from_params(p, rd).to(DEV).requires_grad_(True)
    packed = nat.PackedWeights(mode, rd, DEV)
    packed.pack(flat.detach())
    return p, flat, packed


@pytest.mark.parametrize("contraction", ["aabb", "sphere", "tanh"])
@pytest.mark.parametrize("mode,tol", [("f32", 1e-4), ("bf16", 2e-2)])
def test_field_point_gradients(contraction, mode, tol):
    """points = 1: d(points), d(directions) of sum(g_rgb rgb + g_sigma sigma)."""
    nat = _nat()
    rd, n = 3, 512
    p, flat, packed = _field_setup(mode, rd, 3)
    g = torch.Generator().manual_seed(4)
    span = 1.6 if contraction == "aabb" else 4.0
    x = torch.rand(n, 3, generator=g) * 2 * span - span
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=-1)
    g_rgb, g_sig = torch.randn(n, rd, generator=g), torch.randn(n, generator=g)
    xd, dd = x.to(DEV).requires_grad_(True), d.to(DEV).requires_grad_(True)
    rgb, sig = nat.field(xd, dd, flat, _cfg(mode, rd, contraction), packed)
    ((rgb * g_rgb.to(DEV)).sum() + (sig * g_sig.to(DEV)).sum()).backward()
    ref = {}
    for dt in (torch.float32, torch.float64):
        pr = {k: v.to(dt) for k, v in p.items()}
        xr, dr = x.detach().clone().to(dt).requires_grad_(True), d.detach().clone().to(dt).requires_grad_(True)
        rgb_r, sig_r = onerf.radiance_field(pr, xr, dr, contraction=contraction)
        ((rgb_r * g_rgb.to(dt)).sum() + (sig_r[:, 0] * g_sig.to(dt)).sum()).backward()
        ref[dt] = (xr.grad, dr.grad)
    (x32, d32), (x64, d64) = ref[torch.float32], ref[torch.float64]
    tx, td = (_floor(x32, x64), _floor(d32, d64)) if mode == "f32" else (tol, tol)
    e_x, e_d = norm_rel(xd.grad, x64), norm_rel(dd.grad, d64)
    print(f"[{mode} {contraction}] d points {e_x:.2e} (bound {tx:.2e}), d dirs {e_d:.2e} (bound {td:.2e})")
    assert e_x <= tx and e_d <= td


@pytest.mark.parametrize("mode,tol", [("f32", 1e-4), ("bf16", 2e-2)])
def test_fixed_sampler_ray_gradients(mode, tol):
    """points = 0 (the benchmark's fused sampler): d(rays_o), d(rays_d) of colour / opacity / depth,
    the stratified intervals held constant (nerfacc's are detached)."""
    nat = _nat()
    rd, S, R = 3, 128, 64
    p, flat, packed = _field_setup(mode, rd, 5)
    o, d, u = synthetic_rays(R, seed=6)
    g = torch.Generator().manual_seed(7)
    gc, go, gd = torch.randn(R, rd, generator=g), torch.randn(R, generator=g), torch.randn(R, generator=g)
    bk = torch.full((rd,), 0.7)
    od, dd = o.to(DEV).requires_grad_(True), d.to(DEV).requires_grad_(True)
    c, op, dp = nat.render(od, dd, u.to(DEV), bk.to(DEV), flat, _cfg(mode, rd), packed, S)
    ((c * gc.to(DEV)).sum() + (op * go.to(DEV)).sum() + (dp * gd.to(DEV)).sum()).backward()
    pr = {k: v.double() for k, v in p.items()}
    with torch.no_grad():
        t0, t1 = onerf.stratified_samples(o, d, u, onerf.AABB_CHAIR, 1.43, 6.63, S)
    t0, t1 = t0.double(), t1.double()
    orr, drr = o.double().requires_grad_(True), d.double().requires_grad_(True)
    pos = orr[:, None, :] + drr[:, None, :] * (t0 + t1)[..., None] / 2.0
    rgb, sig = onerf.radiance_field(pr, pos.reshape(-1, 3), drr[:, None, :].expand(R, S, 3).reshape(-1, 3))
    col, opa, dep, _ = onerf.composite(t0, t1, rgb.reshape(R, S, rd), sig.reshape(R, S), bk.double())
    ((col * gc.double()).sum() + (opa * go.double()).sum() + (dep * gd.double()).sum()).backward()
    e_o, e_d = norm_rel(od.grad, orr.grad), norm_rel(dd.grad, drr.grad)
    print(f"[{mode}] d rays_o {e_o:.2e}, d rays_d {e_d:.2e}")
    assert e_o <= tol and e_d <= tol


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("contraction", ["aabb", "sphere"])
def test_packed_sample_ray_gradients(contraction, mode):
    """points = 2 (the packed ray-marching samples of NeRF.forward): per-ray sums over sorted,
    ragged runs of samples (rays with none among them), padding past the real samples.  BF16 (the
    path NeRF.forward takes when tau_r is learnable): the layer-major hidden backward's dz buffers
    (aliased over S0 / S5) feed the per-ray reduce -- 2e-2 against the f64 autograd."""
    nat = _nat()
    rd, R, n = 1, 40, 1000
    p, flat, packed = _field_setup(mode, rd, 8)
    g = torch.Generator().manual_seed(9)
    o = torch.randn(R, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, -3.0])
    d = torch.nn.functional.normalize(torch.randn(R, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 1.0]), dim=-1)
    ri = torch.randint(0, R, (n,), generator=g).sort().values
    ri[ri == 7] = 8  # a ray without samples
    t0 = torch.rand(n, generator=g) * 5 + 0.5
    t1 = t0 + 0.01
    g_rgb, g_sig = torch.randn(n, rd, generator=g), torch.randn(n, generator=g)
    od, dd = o.to(DEV).requires_grad_(True), d.to(DEV).requires_grad_(True)
    rgb, sig = nat.field_packed(od, dd, ri.to(DEV), t0.to(DEV), t1.to(DEV), flat, _cfg(mode, rd, contraction),
                                packed)
    ((rgb * g_rgb.to(DEV)).sum() + (sig * g_sig.to(DEV)).sum()).backward()
    ref = {}
    for dt in (torch.float32, torch.float64):
        pr = {k: v.to(dt) for k, v in p.items()}
        orr, drr = o.detach().clone().to(dt).requires_grad_(True), d.detach().clone().to(dt).requires_grad_(True)
        pos = orr[ri] + drr[ri] * ((t0 + t1).to(dt) / 2.0)[:, None]
        rgb_r, sig_r = onerf.radiance_field(pr, pos, drr[ri], contraction=contraction)
        ((rgb_r * g_rgb.to(dt)).sum() + (sig_r[:, 0] * g_sig.to(dt)).sum()).backward()
        ref[dt] = (orr.grad, drr.grad)
    (o32, d32), (o64, d64) = ref[torch.float32], ref[torch.float64]
    to_, td = (_floor(o32, o64), _floor(d32, d64)) if mode == "f32" else (2e-2, 2e-2)
    e_o, e_d = norm_rel(od.grad, o64), norm_rel(dd.grad, d64)
    print(f"[packed {contraction} {mode}] d rays_o {e_o:.2e} (bound {to_:.2e}), d rays_d {e_d:.2e} (bound {td:.2e})")
    assert e_o <= to_ and e_d <= td
    assert float(od.grad[7].abs().max()) == 0.0


@pytest.mark.parametrize("ctype", [0, 2, 1])
def test_ngp_ray_gradients(ctype):
    """The ngp field's input gradient (tcnn's Linear grid-encoding input gradient, SH, contraction)
    at points and at packed samples, against oracle/ngp.field autograd (f64)."""
    from deblur_e_nerf import _native
    from oracle import ngp as ongp
    rd = 3
    pos = dict(ongp.POS_ENCODING, n_levels=8, log2_hashmap_size=14)
    aabb = [-1.5, -1.5, -1.5, 1.5, 1.5, 1.5]
    p = ongp.build_params(rd, 31, pos, table_scale=0.5)
    desc = _native.ngp_desc(rd, pos, "softplus", "softplus", ctype, aabb)
    names = ["mlp_base.0.params"] + [f"{k}.{t}" for k, _, _ in ongp.layer_specs(rd, pos) for t in ("weight", "bias")]
    flat = torch.cat([p[k].reshape(-1) for k in names]).to(DEV).requires_grad_(True)
    g = torch.Generator().manual_seed(32)
    R, n = 30, 900
    o = torch.randn(R, 3, generator=g) * 0.2
    d = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1)
    ri = torch.randint(0, R, (n,), generator=g).sort().values
    t0 = torch.rand(n, generator=g) * (2.5 if ctype else 1.2)
    t1 = t0 + 0.004
    g_rgb, g_sig = torch.randn(n, rd, generator=g), torch.randn(n, generator=g)
    od, dd = o.to(DEV).requires_grad_(True), d.to(DEV).requires_grad_(True)
    rgb, sig = _native.ngp_field_packed(flat, desc, od, dd, ri.to(DEV), t0.to(DEV), t1.to(DEV))
    ((rgb * g_rgb.to(DEV)).sum() + (sig * g_sig.to(DEV)).sum()).backward()
    pr = {k: v.double() for k, v in p.items()}
    orr, drr = o.double().requires_grad_(True), d.double().requires_grad_(True)
    x = orr[ri] + drr[ri] * ((t0 + t1).double() / 2.0)[:, None]
    rgb_r, sig_r = ongp.field(pr, x, drr[ri], rd, torch.tensor(aabb, dtype=torch.float64), ctype, pos)
    ((rgb_r * g_rgb.double()).sum() + (sig_r[:, 0] * g_sig.double()).sum()).backward()
    e_o, e_d = norm_rel(od.grad, orr.grad), norm_rel(dd.grad, drr.grad)
    print(f"[ngp ctype {ctype}] d rays_o {e_o:.2e}, d rays_d {e_d:.2e}")
    assert e_o <= 1e-4 and e_d <= 1e-4
    # points = 1: per-point gradients
    xp = x.detach().float().to(DEV).requires_grad_(True)
    dp = drr[ri].detach().float().to(DEV).requires_grad_(True)
    rgb, sig = _native.ngp_field(flat, desc, xp, dp)
    ((rgb * g_rgb.to(DEV)).sum() + (sig * g_sig.to(DEV)).sum()).backward()
    xr2, dr2 = x.detach().requires_grad_(True), drr[ri].detach().requires_grad_(True)
    rgb_r, sig_r = ongp.field(pr, xr2, dr2, rd, torch.tensor(aabb, dtype=torch.float64), ctype, pos)
    ((rgb_r * g_rgb.double()).sum() + (sig_r[:, 0] * g_sig.double()).sum()).backward()
    assert norm_rel(xp.grad, xr2.grad) <= 1e-4 and norm_rel(dp.grad, dr2.grad) <= 1e-4


def test_pixel_rays_backward():
    """den_pixel_rays_bwd vs autograd of NeRF.pixel_params_to_ray (oracle/events.py), with a
    leading render-group dim."""
    nat = _nat()
    from oracle import events as oev
    g = torch.Generator().manual_seed(11)
    M, N = 3, 257
    K = torch.tensor([[1111.0, 0.0, 400.0], [0.0, 1111.0, 400.0], [0.0, 0.0, 1.0]])
    kinv = torch.linalg.inv(K)
    pix = torch.rand(N, 2, generator=g) * 799
    pos = torch.randn(M, N, 3, generator=g)
    q = torch.nn.functional.normalize(torch.randn(M * N, 4, generator=g), dim=-1)
    from oracle import roma
    rot = roma.unitquat_to_rotmat(q).reshape(M, N, 3, 3)
    go, gd = torch.randn(M, N, 3, generator=g), torch.randn(M, N, 3, generator=g)
    pd, rdv = pos.to(DEV).requires_grad_(True), rot.to(DEV).requires_grad_(True)
    o, d = nat.pixel_rays(kinv.to(DEV), pix.to(DEV), pd, rdv)
    ((o * go.to(DEV)).sum() + (d * gd.to(DEV)).sum()).backward()
    pr, rr = pos.double().requires_grad_(True), rot.double().requires_grad_(True)
    o_r, d_r = oev.pixel_params_to_ray(kinv.double(), pix.double(), pr, rr)
    ((o_r * go.double()).sum() + (d_r * gd.double()).sum()).backward()
    assert norm_rel(pd.grad, pr.grad) <= 1e-6 and norm_rel(rdv.grad, rr.grad) <= 1e-5


def test_trajectory_backward(golden_dir):
    """den_trajectory_bwd (d query timestamp) vs autograd of the trajectory oracle (pinned
    bit-exact to the reference LinearTrajectory by traj.npz) on the fixture's poses: shortest-path
    flips, a near-identical pair, the first stamp and queries exactly on stamps."""
    nat = _nat()
    from oracle import trajectory as otr
    z = np.load(f"{golden_dir}/traj.npz")
    T, P, Q = (torch.from_numpy(z[k]) for k in ("T_wc_timestamp", "T_wc_position", "T_wc_orientation"))
    qt = torch.from_numpy(z["query_ts"])
    g = torch.Generator().manual_seed(12)
    gp, gr = torch.randn(qt.shape[0], 3, generator=g), torch.randn(qt.shape[0], 3, 3, generator=g)
    qd = qt.to(DEV).requires_grad_(True)
    pos, rot = nat.trajectory(T.to(DEV), P.to(DEV), Q.to(DEV), qd)
    ((pos * gp.to(DEV)).sum() + (rot * gr.to(DEV)).sum()).backward()
    qr = qt.clone().requires_grad_(True)
    p_r, r_r = otr.linear_trajectory(T, P.double(), Q.double(), qr)
    ((p_r * gp.double()).sum() + (r_r * gr.double()).sum()).backward()
    e = norm_rel(qd.grad, qr.grad)
    ew = float(((qd.grad.cpu() - qr.grad).abs() / qr.grad.abs().clamp_min(1e-30)).median())
    print(f"trajectory d t: {e:.2e} tensor-wise, median element {ew:.2e}")
    assert e <= 1e-4


def test_pixbw_timestamp_backward():
    """den_pixbw_sample_ts_bwd (d output_ts = sum over the S samples) and den_pixbw_decay_ts_bwd
    (the offset decay of a non-reset call) vs autograd of the same expressions in f64."""
    nat = _nat()
    g = torch.Generator().manual_seed(13)
    S, N = 16, 300
    gen = torch.full((S - 1, N), 0.5, dtype=torch.float64)
    ots = (torch.rand(N, generator=g, dtype=torch.float64) * 1e8 + 5e8)
    gts = torch.randn(S, N, generator=g, dtype=torch.float64)
    od = ots.to(DEV).requires_grad_(True)
    ts = nat.pixbw_sample_ts(gen.to(DEV), od, 2 * np.pi * 21, 0.95)
    (ts * gts.to(DEV)).sum().backward()
    assert torch.allclose(od.grad.cpu(), gts.sum(0), rtol=1e-12, atol=0)
    # decay: out = y - delta exp(-1e-9 f32(ots - rts) / tau_diff)
    prm = torch.tensor([1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0 / (2 * np.pi * 82000.0)])
    rts = ots - torch.rand(N, generator=g, dtype=torch.float64) * 2e4  # decays of e^0 .. e^-10
    delta = torch.randn(N, generator=g) * 1e-2
    d_out = torch.randn(N, generator=g)
    L = nat.lib()
    d_o = torch.empty(N, dtype=torch.float64, device=DEV)
    d_r = torch.empty(N, dtype=torch.float64, device=DEV)
    dev_in = [t.to(DEV) for t in (ots, rts, prm, delta, d_out)]  # kept alive across the call
    nat._check(L.den_pixbw_decay_ts_bwd(N, *(nat._ptr(t) for t in dev_in), nat._ptr(d_o), nat._ptr(d_r),
                                        nat._stream()))
    torch.cuda.synchronize()
    o64, r64 = ots.clone().requires_grad_(True), rts.clone().requires_grad_(True)
    out = -delta.double() * torch.exp(-(1e-9 * (o64 - r64)) / prm[6].double())
    (out * d_out.double()).sum().backward()
    assert norm_rel(d_o, o64.grad) <= 1e-6 and norm_rel(d_r, r64.grad) <= 1e-6


@pytest.mark.parametrize("has_diff,has_tv", [(True, True), (True, False), (False, True)])
def test_event_prep_backward(has_diff, has_tv):
    """EventPrepFunction's reverse mode (den_event_prep_bwd) vs autograd of the oracle restatement
    of ContrastThreshold / RefractoryPeriod / the supervision timestamps (f64): upstream gradients on
    every output, in particular the render timestamps, where the pose path's gradient enters."""
    nat = _nat()
    from deblur_e_nerf.train import synthetic_events
    from oracle import events as oev
    raw = synthetic_events(500, seed=21)
    g = torch.Generator().manual_seed(22)
    N = raw["end_ts"].numel()
    g_lid = torch.randn(N, generator=g)
    g_start = torch.randn(N, generator=g, dtype=torch.float64)
    g_r = torch.randn(4, N, generator=g, dtype=torch.float64)
    g_d = torch.randn(N, generator=g, dtype=torch.float64)
    g_s = torch.randn(N, generator=g, dtype=torch.float64)
    ct = torch.tensor([0.27, 0.22]).to(DEV).requires_grad_(True)
    tau = torch.tensor([1500.0], dtype=torch.float64).to(DEV).requires_grad_(True)
    args = [raw[k].to(DEV) for k in ("num_pos", "num_neg", "end_ts", "start_ts", "normalized")]
    lid, start, rts, tsd, tss, _ = nat.EventPrepFunction.apply(*args, ct, tau, None, has_diff, has_tv)
    total = (lid * g_lid.to(DEV)).sum() + (start * g_start.to(DEV)).sum()
    if has_diff:
        total = total + (rts[:2] * g_r[:2].to(DEV)).sum() + (tsd * g_d.to(DEV)).sum()
    if has_tv:
        total = total + (rts[2:] * g_r[2:].to(DEV)).sum() + (tss * g_s.to(DEV)).sum()
    total.backward()
    ctr = torch.tensor([0.27, 0.22], dtype=torch.float64, requires_grad=True)
    taur = torch.tensor(1500.0, dtype=torch.float64, requires_grad=True)
    o = oev.event_prep(raw["num_pos"], raw["num_neg"], raw["end_ts"], raw["start_ts"], raw["normalized"], ctr[0],
                       ctr[1], taur, has_diff, has_tv)
    tot = (o["lid"] * g_lid.double()).sum() + (o["start_ts"] * g_start).sum()
    if has_diff:
        dt, s, e = o["diff"]
        tot = tot + (s * g_r[0]).sum() + (e * g_r[1]).sum() + (dt * g_d).sum()
    if has_tv:
        dt, s, e = o["subdiff"]
        tot = tot + (s * g_r[2]).sum() + (e * g_r[3]).sum() + (dt * g_s).sum()
    tot.backward()
    assert norm_rel(ct.grad, ctr.grad) <= 1e-6
    assert abs(float(tau.grad) - float(taur.grad)) <= 1e-9 * abs(float(taur.grad))
