"""Pin the CPU oracle against golden vectors produced by the reference's own
modules (tests/golden/make_golden.py).  CPU only."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import loss as oloss
from oracle import nerf as onerf
from oracle import pixbw as opb


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))


# --------------------------------------------------------------------------- radiance field
@pytest.mark.parametrize("fixture,rd", [("mlp_rd1", 1), ("mlp_rd3", 3), ("mlp_rd3_sphere", 3), ("mlp_rd1_tanh", 1),
                                        ("mlp_rd1_shifted_softplus", 1), ("mlp_rd3_softplus", 3)])
def test_radiance_field_matches_reference(golden_dir, fixture, rd):
    z = _load(golden_dir, fixture + ".npz")
    contraction = str(z["contraction"]) if "contraction" in z.files else "aabb"
    density = str(z["density"]) if "density" in z.files else "shifted_trunc_exp"
    p = onerf.build_params(rd, int(z["seed"]))
    # same weights as the reference's construction under the same seed
    for name in z["param_names"]:
        assert abs(p[str(name)].double().sum().item() - float(z[f"wsum:{name}"])) < 1e-9 * max(1, abs(float(z[f"wsum:{name}"]))) + 1e-6
    for k in p:
        p[k].requires_grad_(True)
    x = torch.from_numpy(z["x"])
    d = torch.from_numpy(z["d"])
    rgb, sig = onerf.radiance_field(p, x, d, contraction=contraction, density=density)
    # bitwise-level agreement with the reference's fp32 forward (same torch ops on CPU)
    assert rel_err(rgb.detach(), z["rgb_f32"]) < 1e-6
    assert rel_err(sig.detach(), z["sigma_f32"]) < 1e-6
    # and the reference's own fp32-vs-fp64 gap is small too
    assert rel_err(z["rgb_f32"], z["rgb_f64"]) < 1e-5
    ((rgb * torch.from_numpy(z["g_rgb"])).sum() + (sig * torch.from_numpy(z["g_sigma"])).sum()).backward()
    for name in z["param_names"]:
        name = str(name)
        g = p[name].grad.numpy().astype(np.float64)
        ref_norm = float(z[f"gnorm_f32:{name}"])
        assert abs(np.linalg.norm(g) - ref_norm) <= 1e-5 * max(ref_norm, 1e-6) + 1e-9, name
        if f"grad:{name}" in z.files:
            ref = z[f"grad:{name}"]
            scale = max(np.abs(ref).max(), 1e-6)
            assert np.abs(g - ref).max() <= 1e-5 * scale, name


def test_encoding_layout():
    v = torch.tensor([[0.1, -0.2, 0.3]])
    e = onerf.encode(v, 2)
    # [v, sin(v), sin(2v), cos(v), cos(2v)] scale-major / dim-minor
    exp = [0.1, -0.2, 0.3] + [math.sin(a) for a in (0.1, -0.2, 0.3, 0.2, -0.4, 0.6)] \
        + [math.cos(a) for a in (0.1, -0.2, 0.3, 0.2, -0.4, 0.6)]
    assert np.allclose(e.numpy()[0], exp, atol=1e-6)


def test_trunc_exp_backward_clamp():
    x = torch.tensor([0.0, 10.0, 20.0], requires_grad=True)
    y = onerf._TruncExp.apply(x)
    y.sum().backward()
    assert torch.allclose(x.grad, torch.exp(torch.tensor([0.0, 10.0, 15.0])))


# --------------------------------------------------------------------------- compositing (unpinned)
def test_composite_vs_bruteforce():
    g = torch.Generator().manual_seed(0)
    R, N, rd = 5, 37, 3
    t0 = torch.sort(torch.rand(R, N, generator=g) * 4 + 1, dim=-1).values
    t1 = t0 + torch.rand(R, N, generator=g) * 0.05
    rgb = torch.rand(R, N, rd, generator=g)
    sig = torch.rand(R, N, generator=g) * 30
    bk = torch.tensor([0.3, 0.5, 0.7])
    c, o, dpt, _ = onerf.composite(t0, t1, rgb, sig, bk)
    c2, o2, d2 = onerf.composite_bruteforce_f64(t0, t1, rgb, sig, bk)
    assert rel_err(c, c2) < 1e-5 and rel_err(o, o2) < 1e-5 and rel_err(dpt, d2) < 1e-5


def test_sampler_strata_and_miss():
    o = torch.tensor([[0.0, 0.0, -4.0], [0.0, 5.0, -4.0]])
    d = torch.tensor([[0.0, 0.0, 1.0], [0.0, 0.0, 1.0]])
    u = torch.tensor([0.25, 0.5])
    t0, t1 = onerf.stratified_samples(o, d, u, onerf.AABB_CHAIR, 1.43, 6.63, 8)
    mid = (t0 + t1) / 2
    # ray 0 crosses the box on z in [2.5, 5.5]
    assert torch.allclose(mid[0], 2.5 + (torch.arange(8) + 0.25) / 8 * 3.0)
    assert torch.allclose(t1[0] - t0[0], torch.full((8,), 3.0 / 8))
    # ray 1 misses the box: zero-width intervals -> zero weights
    assert torch.all(t1[1] == t0[1])


# --------------------------------------------------------------------------- FOH
def test_foh_matches_reference(golden_dir):
    z = _load(golden_dir, "foh.npz")
    for tag, dt_ in (("f64", torch.float64), ("f32", torch.float32)):
        A = torch.from_numpy(z["A"]).to(dt_)
        B = torch.from_numpy(z["B"]).to(dt_)
        dt = torch.from_numpy(z["dt"]).to(dt_)
        Ad, Bd, Btd = opb.foh_discretise(A, B, dt)
        tol = 1e-12 if tag == "f64" else 1e-5
        assert rel_err(Ad, z[f"Ad_{tag}_eff"]) < tol
        assert rel_err(Bd, z[f"Bd_{tag}_eff"]) < tol
        assert rel_err(Btd, z[f"Btd_{tag}_eff"]) < tol
    # efficient vs block-expm agree in the reference itself (f64)
    assert rel_err(z["Ad_f64_eff"], z["Ad_f64_blk"]) < 1e-9


# --------------------------------------------------------------------------- pixel bandwidth
def _intensity_of(ts, z):
    t = ts * 1e-9
    base, amp, freq, phase = (torch.from_numpy(z[k]) for k in ("base", "amp", "freq", "phase"))
    return base * torch.exp(amp * torch.sin(2 * np.pi * freq * t + phase))


@pytest.mark.parametrize("fname", ["pixbw_S16_eds.npz", "pixbw_S30_eds.npz", "pixbw_S16_pert.npz"])
def test_pixel_bandwidth_matches_reference(golden_dir, fname):
    z = _load(golden_dir, fname)
    calib = {k.split(":", 1)[1]: z[k] for k in z.files if k.startswith("calib:")}
    base_prm = opb.calib_to_params(calib)
    call_ts = torch.from_numpy(z["call_ts"])
    coef = torch.from_numpy(z["coef"])
    for gi, gname in enumerate(("gen_dirac", "gen_unif")):
        gen = torch.from_numpy(z[gname])
        for dtag, dtype in (("f32", torch.float32), ("f64", torch.float64)):
            # parameters exactly as the module holds them: softplus(original)
            originals = {}
            prm = {"tau_in_it_eff_prod": torch.tensor(np.float32(base_prm["tau_in_it_eff_prod"])).to(dtype)}
            for pn in opb.PARAM_NAMES:
                orig = torch.tensor(z[f"orig_{dtag}:{pn}"], dtype=dtype).requires_grad_(True)
                originals[pn] = orig
                prm[pn] = torch.nn.functional.softplus(orig, beta=1, threshold=20)
            pb = opb.PixelBandwidthOracle(prm, int(z["min_ts"]))
            leaves = []

            def fn(ts):
                it = _intensity_of(ts, z).to(dtype).detach().requires_grad_(True)
                leaves.append(it)
                return it

            outs = [pb(gen, call_ts[c], fn, reset_diff=(c == 0)) for c in range(4)]
            total = sum((outs[c] * coef[c].to(dtype)).sum() for c in range(4))
            total.backward()
            tol = 1e-7 if dtag == "f64" else 2e-6
            for c in range(4):
                assert rel_err(outs[c].detach(), z[f"logit_g{gi}_{dtag}_c{c}"]) < tol, (c, dtag)
                ref = z[f"dit_g{gi}_{dtag}_c{c}"]
                assert np.abs(leaves[c].grad.numpy() - ref).max() <= (1e-6 if dtag == "f64" else 1e-3) * np.abs(ref).max()
            for pn in opb.PARAM_NAMES:
                ref = z[f"dparam_g{gi}_{dtag}:{pn}"]
                got = originals[pn].grad.numpy()
                assert abs(got - ref) <= (1e-6 if dtag == "f64" else 2e-3) * max(abs(ref), 1e-30), (pn, dtag)


# --------------------------------------------------------------------------- loss / event model
@pytest.mark.parametrize("t", ["huber_l1", "l1_huber", "mse_mse", "mape_l1"])
def test_loss_matches_reference(golden_dir, t):
    z = _load(golden_dir, "loss.npz")
    fd, ft = t.split("_")
    d_lid = torch.from_numpy(z[f"{t}:d_lid"]).requires_grad_(True)
    s_lid = torch.from_numpy(z[f"{t}:s_lid"]).requires_grad_(True)
    mct = torch.tensor(0.225, requires_grad=True)
    end_ts = torch.from_numpy(z[f"{t}:end_ts"])
    start_ts = torch.from_numpy(z[f"{t}:start_ts"])
    Ld, Lt = oloss.event_loss(torch.from_numpy(z[f"{t}:lid"]), end_ts, start_ts, d_lid,
                              (end_ts - start_ts) * 1.0, torch.from_numpy(z[f"{t}:d_valid"]),
                              s_lid, torch.from_numpy(z[f"{t}:s_valid"]), mct, fd, ft)
    assert rel_err(Ld.detach(), z[f"{t}:L_diff"]) < 1e-6
    assert rel_err(Lt.detach(), z[f"{t}:L_tv"]) < 1e-6
    (Ld + 1e-3 * Lt).backward()
    assert np.abs(d_lid.grad.numpy() - z[f"{t}:g_d_lid"]).max() < 1e-9
    assert np.abs(s_lid.grad.numpy() - z[f"{t}:g_s_lid"]).max() < 1e-9
    assert rel_err(mct.grad.numpy(), z[f"{t}:g_mct"]) < 1e-5


def test_contrast_threshold_matches_reference(golden_dir):
    z = _load(golden_dir, "ct.npz")
    lid = oloss.contrast_log_intensity_diff(torch.from_numpy(z["num_pos"]), torch.from_numpy(z["num_neg"]),
                                            torch.from_numpy(z["pos_ct"]), torch.from_numpy(z["neg_ct"]))
    assert np.array_equal(lid.numpy(), z["lid"])


# --------------------------------------------------------------------------- event preparation / pixel rays
@pytest.mark.parametrize("tag,has_diff,has_tv", [("both", True, True), ("diff", True, False), ("tv", False, True)])
def test_event_prep_matches_reference(golden_dir, tag, has_diff, has_tv):
    """events.npz = the reference's ContrastThreshold / RefractoryPeriod modules
    and its training_step timestamp block, run here: the oracle is bit-exact."""
    from oracle import events as oev
    z = _load(golden_dir, "events.npz")
    t = {k: torch.from_numpy(z[k]) for k in ("num_pos", "num_neg", "end_ts", "start_ts", "norm", "pos_ct", "neg_ct",
                                               "refractory_period")}
    o = oev.event_prep(t["num_pos"], t["num_neg"], t["end_ts"], t["start_ts"], t["norm"], t["pos_ct"], t["neg_ct"],
                       t["refractory_period"], has_diff, has_tv)
    assert o["lid"].dtype == torch.float32 and o["start_ts"].dtype == torch.float64
    assert np.array_equal(o["lid"].numpy(), z[f"{tag}:lid"])
    assert np.array_equal(o["start_ts"].numpy(), z[f"{tag}:start_ts"])
    for grp, have in (("diff", has_diff), ("subdiff", has_tv)):
        assert (o[grp] is not None) == have
        if have:
            for i, k in enumerate(("ts_diff", "start_ts", "end_ts")):
                assert np.array_equal(o[grp][i].numpy(), z[f"{tag}:{grp}.{k}"]), (grp, k)


def test_pixel_rays_match_reference(golden_dir):
    from oracle import events as oev
    z = _load(golden_dir, "rays.npz")
    K, px, pos, rot = (torch.from_numpy(z[k]) for k in ("K_inv", "pixel", "T_wc_position", "T_wc_orientation"))
    o, d = oev.pixel_params_to_ray(K, px, pos, rot)
    assert np.array_equal(o.numpy(), z["ray_origin"])
    assert rel_err(d, z["ray_direction"]) < 1e-7
    o1, d1 = oev.pixel_params_to_ray(K, px, pos[0], rot[0])
    assert rel_err(d1, z["ray_direction_1"]) < 1e-7
    assert np.allclose(np.linalg.norm(z["ray_direction"], axis=-1), 1.0, atol=1e-6)


# --------------------------------------------------------------------------- ngp radiance field
NGP_FIXTURES = ["ngp_rd1_small", "ngp_rd3_small_sphere_relu_sigmoid", "ngp_rd3_small_tanh", "ngp_rd3_default",
                "ngp_rd1_small_shifted_softplus", "ngp_rd3_small_sphere_softplus"]


@pytest.mark.parametrize("fixture", NGP_FIXTURES)
def test_ngp_field_matches_reference(golden_dir, fixture):
    """oracle/ngp.py (contraction, SH, MLPs, activations around oracle/tcnn.py) against the
    reference's NGPradianceField run with the same encoding: outputs 1e-6, gradients 1e-5."""
    from _util import ngp_fixture, ngp_table_grad
    from oracle import ngp as ongp
    z = _load(golden_dir, fixture + ".npz")
    p, pos, base, head, rd, ctype = ngp_fixture(z)
    for k in p:
        p[k].requires_grad_(True)
    rgb, sig = ongp.field(p, torch.from_numpy(z["x"]), torch.from_numpy(z["d"]), rd, torch.from_numpy(z["aabb"]),
                          ctype, pos, base, head)
    assert rel_err(rgb.detach(), z["rgb"]) < 1e-6 and rel_err(sig.detach(), z["sigma"]) < 1e-6
    ((rgb * torch.from_numpy(z["g_rgb"])).sum() + (sig * torch.from_numpy(z["g_sigma"])).sum()).backward()
    for k, v in p.items():
        ref = ngp_table_grad(z, v.numel()) if k == "mlp_base.0.params" else torch.from_numpy(z[f"grad:{k}"])
        e = (v.grad - ref).abs().max().item() / max(ref.abs().max().item(), 1e-12)
        assert e < 1e-5, (k, e)


def test_tcnn_grid_levels_follow_tcnn_sizing():
    """synthetic.yaml's HashGrid: level 0..4 dense (res 16, 24, 34, 49, 71 -> entries rounded to 8),
    levels 5..15 hashed at 2^19: 6,299,960 entries x 2 = 12,599,920 parameters."""
    from oracle import ngp as ongp
    from oracle import tcnn as otcnn
    c = ongp.POS_ENCODING
    levels, total = otcnn.grid_levels(c["n_levels"], c["log2_hashmap_size"], c["base_resolution"],
                                      c["per_level_scale"])
    res = [r for _, r, _, _ in levels]
    assert res[:5] == [16, 24, 34, 49, 71]
    assert [e for _, _, e, _ in levels[:5]] == [4096, 13824, 39304, 117656, 357912]
    assert all(e == 1 << 19 for _, _, e, _ in levels[5:])
    assert total * 2 == otcnn.n_params(c) == 12599920


def test_trajectory_oracle_matches_reference(golden_dir):
    """oracle/trajectory.linear_trajectory (the differentiable restatement the trajectory-backward
    tests check against) reproduces the reference LinearTrajectory's outputs (traj.npz) exactly."""
    from oracle import trajectory as otr
    z = np.load(os.path.join(golden_dir, "traj.npz"))
    T, P, Q = (torch.from_numpy(z[k]) for k in ("T_wc_timestamp", "T_wc_position", "T_wc_orientation"))
    for q, kp, kr in (("query_ts", "position", "rotation"), ("query_ts_2d", "position_2d", "rotation_2d")):
        p, r = otr.linear_trajectory(T, P, Q, torch.from_numpy(z[q]))
        assert torch.equal(p, torch.from_numpy(z[kp])) and torch.equal(r, torch.from_numpy(z[kr]))


@pytest.mark.parametrize("degree", range(1, 9))
def test_sh_oracle_matches_reference(golden_dir, degree):
    """oracle/sh.py (Legendre-derivative restatement) vs the reference SHEncoder's outputs and autograd
    gradients (make_golden.gen_sh), degrees 1..8, unit and non-unit coords: f32 rounding only."""
    from oracle import sh as osh
    z = _load(golden_dir, "sh_encoder.npz")
    out = osh.sh_encode(z["coords"], degree)
    ref = z[f"out_{degree}"]
    assert np.abs(out - ref).max() <= 1e-6 * np.abs(ref).max()
    g = osh.sh_encode_grad(z["coords"], degree, z[f"g_{degree}"])
    gref = z[f"dcoords_{degree}"]
    assert np.abs(g - gref).max() <= 1e-6 * max(np.abs(gref).max(), 1.0)
