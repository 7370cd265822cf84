"""Event preparation (den_event_prep: ContrastThreshold + RefractoryPeriod +
training_step timestamps + diff target) and pixel rays (den_pixel_rays:
NeRF.pixel_params_to_ray) on the GPU, through the C ABI, against the reference's
own outputs (tests/golden/events.npz, rays.npz) and the CPU oracle.

Tolerances: lid (f32) and the refractory-shifted start (f64) are bit-exact; the
lerp'd timestamps are bit-exact too (same fused form as torch's CPU lerp) -- the
test allows 1 ulp of f64 (2^-52 relative, i.e. <0.25 ns at 1e9 ns) in case a
reduction order differs.  Ray directions: 1e-6 relative (f32, 3x3 products).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _golden(golden_dir, name):
    import os
    return np.load(os.path.join(golden_dir, name))


def _ulp_close(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= np.abs(b) * 2.0 ** -52)


@pytest.mark.parametrize("tag,has_diff,has_tv", [("both", 1, 1), ("diff", 1, 0), ("tv", 0, 1)])
def test_event_prep_matches_reference(golden_dir, tag, has_diff, has_tv):
    from deblur_e_nerf import _native as nat
    z = _golden(golden_dir, "events.npz")
    g = {k: torch.from_numpy(z[k]).to(DEV) for k in ("num_pos", "num_neg", "end_ts", "start_ts", "norm")}
    ct = torch.tensor([float(z["pos_ct"]), float(z["neg_ct"])], dtype=torch.float32, device=DEV)
    tau = torch.tensor([float(z["refractory_period"])], dtype=torch.float64, device=DEV)
    c = torch.tensor([float(z["mean_ct"])], device=DEV)
    o = nat.event_prep(g["num_pos"], g["num_neg"], g["end_ts"], g["start_ts"], g["norm"].contiguous(), ct, tau,
                       norm_c=c if has_diff else None, has_diff=has_diff, has_tv=has_tv)
    torch.cuda.synchronize()
    assert np.array_equal(o["lid"].cpu().numpy(), z[f"{tag}:lid"])
    assert np.array_equal(o["start_ts"].cpu().numpy(), z[f"{tag}:start_ts"])
    rts = o["render_ts"].cpu().numpy()
    if has_diff:
        assert _ulp_close(o["ts_diff"].cpu(), z[f"{tag}:diff.ts_diff"])
        assert _ulp_close(rts[0], z[f"{tag}:diff.start_ts"]) and _ulp_close(rts[1], z[f"{tag}:diff.end_ts"])
        # loss.py:74-77 target, f64 arithmetic rounded to f32
        lid = torch.from_numpy(z[f"{tag}:lid"]).double()
        ref_t = (torch.from_numpy(z[f"{tag}:diff.ts_diff"]) * (lid / (torch.from_numpy(z["end_ts"]).double()
                 - torch.from_numpy(z[f"{tag}:start_ts"]))) / float(z["mean_ct"])).float()
        assert torch.allclose(o["target"].cpu(), ref_t, rtol=1e-6, atol=0)
    if has_tv:
        assert _ulp_close(o["ts_subdiff"].cpu(), z[f"{tag}:subdiff.ts_diff"])
        assert _ulp_close(rts[2], z[f"{tag}:subdiff.start_ts"]) and _ulp_close(rts[3], z[f"{tag}:subdiff.end_ts"])
    # interval invariants of the derivation (deblur_e_nerf.py:427-433)
    end = z["end_ts"].astype(np.float64)
    assert np.all(rts[0] >= z[f"{tag}:start_ts"]) if has_diff else True
    assert np.all(rts[1] <= end) if has_diff else True


def test_event_prep_large_random_matches_oracle():
    """2^17 events (the bench's 4 x 32768 render timestamps), random counts and
    samples: bit-exact lid / start, <= 1 ulp timestamps vs the oracle."""
    from deblur_e_nerf import _native as nat
    from oracle import events as oev
    g = torch.Generator().manual_seed(3)
    N = 1 << 17
    num_pos = torch.randint(0, 4, (N,), generator=g)
    num_neg = torch.randint(0, 4, (N,), generator=g)
    end = (torch.rand(N, generator=g, dtype=torch.float64) * 9e8 + 1e8).long()
    start = end - (torch.rand(N, generator=g, dtype=torch.float64) * 5e6 + 2e5).long()
    norm = torch.rand(4, N, generator=g, dtype=torch.float64)
    pc, nc, tau = torch.tensor(0.31), torch.tensor(0.27), torch.tensor(123456.789, dtype=torch.float64)
    r = oev.event_prep(num_pos, num_neg, end, start, norm, pc, nc, tau)
    o = nat.event_prep(num_pos.to(DEV), num_neg.to(DEV), end.to(DEV), start.to(DEV), norm.to(DEV),
                       torch.stack([pc, nc]).to(DEV), tau.reshape(1).to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(o["lid"].cpu(), r["lid"])
    assert torch.equal(o["start_ts"].cpu(), r["start_ts"])
    rts = o["render_ts"].cpu()
    for a, b in ((rts[0], r["diff"][1]), (rts[1], r["diff"][2]), (rts[2], r["subdiff"][1]), (rts[3], r["subdiff"][2]),
                 (o["ts_diff"].cpu(), r["diff"][0]), (o["ts_subdiff"].cpu(), r["subdiff"][0])):
        assert _ulp_close(a, b)


def test_pixel_rays_match_reference(golden_dir):
    from deblur_e_nerf.models.nerf import NeRF
    z = _golden(golden_dir, "rays.npz")
    K, px, pos, rot = (torch.from_numpy(z[k]).to(DEV) for k in ("K_inv", "pixel", "T_wc_position",
                                                                  "T_wc_orientation"))
    o, d = NeRF.pixel_params_to_ray(K, px, pos, rot)
    o1, d1 = NeRF.pixel_params_to_ray(K, px, pos[0].contiguous(), rot[0].contiguous())
    torch.cuda.synchronize()
    assert np.array_equal(o.cpu().numpy(), z["ray_origin"])
    for a, b in ((d, z["ray_direction"]), (d1, z["ray_direction_1"])):
        a = a.cpu().numpy().astype(np.float64)
        assert np.max(np.abs(a - b)) <= 1e-6, np.max(np.abs(a - b))


def test_event_modules_forward():
    """The module mirrors run the same kernel and keep their own outputs."""
    from deblur_e_nerf.models.event_generation_params import ContrastThreshold, RefractoryPeriod
    cal = dict(pos_contrast_threshold=np.float32(0.25), neg_contrast_threshold=np.float32(0.2),
               refractory_period=np.int64(250000))
    ctm = ContrastThreshold(calibration=cal, parameterize_mean_ct=True)
    rpm = RefractoryPeriod(calibration=cal, max_refractory_period=torch.tensor(1000000))
    g = torch.Generator().manual_seed(4)
    N = 1000
    ev = dict(num_pos=torch.randint(0, 3, (N,), generator=g), num_neg=torch.randint(0, 3, (N,), generator=g),
              end_ts=torch.randint(10**8, 10**9, (N,), generator=g))
    ev["start_ts"] = ev["end_ts"] - 10**6
    dev_ev = {k: v.to(DEV) for k, v in ev.items()}
    o = rpm(ctm(dev_ev))
    torch.cuda.synchronize()
    lid_ref = ev["num_pos"] * ctm.pos_contrast_threshold.detach() - ev["num_neg"] * ctm.neg_contrast_threshold.detach()
    assert torch.equal(o["log_intensity_diff"].cpu(), lid_ref.float())
    assert torch.equal(o["start_ts"].cpu(), ev["start_ts"] + rpm.refractory_period.detach())


def test_event_prep_rejects_bad_input():
    from deblur_e_nerf import _native as nat
    x = torch.zeros(8, dtype=torch.int64, device=DEV)
    with pytest.raises(nat.DenError):
        nat.event_prep(x, x, x, x.double(), torch.zeros(4, 8, dtype=torch.float64, device=DEV),
                       torch.zeros(2, device=DEV), torch.zeros(1, dtype=torch.float64, device=DEV))
    with pytest.raises(nat.DenError):
        nat.pixel_rays(torch.eye(3, device=DEV), torch.zeros(5, 2, device=DEV), torch.zeros(4, 6, 3, device=DEV),
                       torch.zeros(4, 6, 3, 3, device=DEV))


@pytest.mark.parametrize("t", ["huber_l1", "l1_huber", "mse_mse", "mape_l1"])
def test_loss_kernels_match_reference(golden_dir, t):
    """loss_metric.Loss.compute on the device (den_event_target + den_event_loss_fwd/bwd) against the
    reference's Loss (loss.npz, make_golden.gen_loss: loss.py:34-96 with utils/modules.py's MAPELoss):
    both loss terms and the gradients into the rendered differences and the mean contrast
    threshold (the normaliser and the target's 1 / C)."""
    from deblur_e_nerf.loss_metric.loss import Loss
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    z = _golden(golden_dir, "loss.npz")
    fd, ft = t.split("_")
    L = Loss(ED(log_intensity_diff=1.0, log_intensity_tv=1e-3), ED(log_intensity_diff=fd, log_intensity_tv=ft),
             ED(log_intensity_diff=True, log_intensity_tv=True))
    d_lid = torch.from_numpy(z[f"{t}:d_lid"]).to(DEV).requires_grad_(True)
    s_lid = torch.from_numpy(z[f"{t}:s_lid"]).to(DEV).requires_grad_(True)
    mct = torch.tensor(0.225, device=DEV, requires_grad=True)
    end_ts = torch.from_numpy(z[f"{t}:end_ts"]).to(DEV)
    start_ts = torch.from_numpy(z[f"{t}:start_ts"]).to(DEV)
    be = ED(log_intensity_diff=torch.from_numpy(z[f"{t}:lid"]).to(DEV), end_ts=end_ts, start_ts=start_ts)
    bd = ED(log_intensity_diff=d_lid, ts_diff=(end_ts - start_ts) * 1.0,
            is_valid=torch.from_numpy(z[f"{t}:d_valid"]).to(DEV))
    bs = ED(log_intensity_diff=s_lid, is_valid=torch.from_numpy(z[f"{t}:s_valid"]).to(DEV))
    res = L.compute(be, bd, bs, mct)
    (res.log_intensity_diff * 1.0 + res.log_intensity_tv * 1e-3).backward()
    torch.cuda.synchronize()
    rel = lambda a, b: float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))  # noqa: E731
    e = {"L_diff": rel(float(res.log_intensity_diff), z[f"{t}:L_diff"]),
         "L_tv": rel(float(res.log_intensity_tv), z[f"{t}:L_tv"]),
         "g_d_lid": rel(d_lid.grad.cpu().numpy(), z[f"{t}:g_d_lid"]),
         "g_s_lid": rel(s_lid.grad.cpu().numpy(), z[f"{t}:g_s_lid"]),
         "g_mct": rel(float(mct.grad), z[f"{t}:g_mct"])}
    print(f"[{t}] {e}")
    assert max(e["L_diff"], e["L_tv"], e["g_d_lid"], e["g_s_lid"]) <= 1e-5, e
    assert e["g_mct"] <= 1e-4, e  # a sum of cancelling terms (the normaliser vs the target's 1 / C)
