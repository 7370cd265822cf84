"""Oracle: one training step of the synthetic configuration (pixel bandwidth off)
-- CPU PyTorch restatement (test infrastructure, see oracle/__init__.py).

Follows DeblurENeRF.training_step (deblur_e_nerf.py:472-586) for
pixel_bandwidth.enable = false: 4 renders (diff start/end, TV start/end) of N
events, I = radiance + min_modeled_intensity (:1200), y = log I (:1158),
Huber diff + L1 TV losses (loss.py:34-96), total = w_d L_diff + w_t L_tv
(:539-545), then torch.optim.Adam with L2 weight decay on the MLP parameters
(:1055-1112).
"""
import torch

from . import loss as oloss
from . import nerf as onerf


def step_loss(p, bkgd, batch, n_samples, w=(1.0, 1e-3), min_int=1e-3, mean_ct=0.25, fn=("huber", "l1")):
    """-> (total, L_diff, L_tv) for the batch layout of deblur_e_nerf.train.synthetic_batch."""
    N = batch["lid"].numel()
    col, op, _, _ = onerf.render_rays(p, batch["rays_o"], batch["rays_d"], batch["jitter"], n_samples=n_samples,
                                      bkgd=bkgd)
    if batch.get("channel") is not None:  # bayering (deblur_e_nerf.py:1223-1235): one channel per event
        ch = batch["channel"].long().repeat(4)[:, None]
        rad = col.gather(1, ch)[:, 0]
    else:
        rad = col[:, 0]
    y = torch.log(rad + min_int).view(4, N)
    if bkgd is None:
        valid = (op > 0).view(4, N)
        vd, vt = valid[0] | valid[1], valid[2] | valid[3]
    else:
        vd = vt = torch.ones(N, dtype=torch.bool)
    c = torch.tensor(mean_ct)
    Ld, Lt = oloss.event_loss(batch["lid"], batch["end_ts"], batch["start_ts"], y[1] - y[0], batch["ts_diff"], vd,
                              y[3] - y[2], vt, c, fn_diff=fn[0], fn_tv=fn[1])
    return w[0] * Ld + w[1] * Lt, Ld, Lt


def flat_grad(p, bkgd_raw, batch, n_samples, rd, **kw):
    """Gradient of the step loss w.r.t. the flat [MLP params | bkgd] vector (the
    TrainStep gradient-buffer layout: d/d softplus(bkgd_raw) last), plus the loss terms."""
    names = [n for n, _, _ in onerf.layer_specs(rd)]
    leaves = []
    for n in names:
        leaves += [p[n + ".weight"], p[n + ".bias"]]
    for t in leaves:
        t.requires_grad_(True)
        t.grad = None
    # the gradient is taken w.r.t. the post-softplus background, as TrainStep's buffer holds it
    bk = torch.nn.functional.softplus(bkgd_raw).detach().requires_grad_(True)
    total, Ld, Lt = step_loss(p, bk, batch, n_samples, **kw)
    total.backward()
    g = torch.cat([t.grad.reshape(-1) for t in leaves] + [bk.grad.reshape(-1)])
    return g.detach(), (float(Ld.detach()), float(Lt.detach()), float(total.detach()))


def prepare_batch(raw, contrast_thresholds=(0.25, 0.25), refractory_period=0.0):
    """Raw event batch (deblur_e_nerf.train.synthetic_events layout) -> the
    prepared layout step_loss consumes, through the oracle's event preparation
    and pixel rays (oracle/events.py)."""
    from . import events as oev
    pc, nc = (torch.tensor(c, dtype=torch.float32) for c in contrast_thresholds)
    o = oev.event_prep(raw["num_pos"], raw["num_neg"], raw["end_ts"], raw["start_ts"], raw["normalized"], pc, nc,
                       torch.tensor(refractory_period, dtype=torch.float64))
    ro, rdir = oev.pixel_params_to_ray(raw["intrinsics_inverse"], raw["position"], raw["T_wc_position"],
                                       raw["T_wc_orientation"])
    return dict(rays_o=ro.reshape(-1, 3), rays_d=rdir.reshape(-1, 3), jitter=raw["jitter"], lid=o["lid"],
                end_ts=raw["end_ts"], start_ts=o["start_ts"], ts_diff=o["diff"][0])


def pixbw_step_loss(p, bkgd, raw, it_sample_size, n_samples, prm, min_ts, w=(1.0, 1e-3), min_int=1e-3, mean_ct=0.25,
                    fn=("huber", "l1"), dt_dtype=torch.float32):
    """The pixel-bandwidth-on step (deblur_e_nerf.train.PixbwTrainStep layout):
    event preparation, then for each supervision timestamp group the S sample
    timestamps, the trajectory's poses (oracle/trajectory.py), rays, renders and the pixel-bandwidth
    filter (oracle/pixbw.py, reset on the diff start), then the losses
    (deblur_e_nerf.py:472-549 with render_log_intensity :1137-1151)."""
    from . import events as oev
    from . import pixbw as opb
    S, N = it_sample_size, raw["end_ts"].numel()
    c = torch.tensor(mean_ct)
    o = oev.event_prep(raw["num_pos"], raw["num_neg"], raw["end_ts"], raw["start_ts"], raw["normalized"], c, c,
                       torch.tensor(0.0, dtype=torch.float64))
    ts_diff, d_s, d_e = o["diff"]
    _, s_s, s_e = o["subdiff"]
    grad = o["lid"] / (raw["end_ts"] - o["start_ts"])
    target = (ts_diff * grad / c).to(torch.float32)
    orc = opb.PixelBandwidthOracle(prm, min_ts, dt_dtype=dt_dtype)
    from . import trajectory as otraj
    jit = raw["jitter"].reshape(4, S * N)
    ys = []
    for g, tg in enumerate((d_s, d_e, s_s, s_e)):
        def intensity(ts, g=g):
            with torch.no_grad():  # tau_r frozen: no gradient through the poses
                pos, rot = otraj.linear_trajectory(raw["T_wc_timestamp"], raw["T_wc_position"].float(),
                                                   raw["T_wc_orientation"].float(), ts.detach())
            # the rays in the poses' precision (f32, as the HIP path's den_pixel_rays); the f64 oracle
            # promotes them below
            ro, rdir = oev.pixel_params_to_ray(raw["intrinsics_inverse"].to(pos.dtype), raw["position"].to(pos.dtype),
                                               pos, rot)
            col, _, _, _ = onerf.render_rays(p, ro.reshape(-1, 3).to(bkgd.dtype), rdir.reshape(-1, 3).to(bkgd.dtype),
                                             jit[g].to(bkgd.dtype), n_samples=n_samples, bkgd=bkgd)
            if raw.get("channel") is not None:
                ch = raw["channel"].long().view(1, N, 1).expand(S, N, 1)
                rad = col.view(S, N, -1).gather(2, ch)[..., 0]
            else:
                rad = col[:, 0].view(S, N)
            return rad + min_int
        ys.append(orc(raw["interval_gen"], tg, intensity, reset_diff=(g == 0)))
    cc = c.to(ys[0].dtype)
    Ld = oloss.ERROR_FNS[fn[0]]((ys[1] - ys[0]) / cc, target.to(ys[0].dtype)).mean()
    Lt = oloss.ERROR_FNS[fn[1]]((ys[3] - ys[2]) / cc, torch.zeros_like(ys[0])).mean()
    return w[0] * Ld + w[1] * Lt, Ld, Lt


def pixbw_flat_grad(p, bkgd_raw, raw, it_sample_size, n_samples, rd, prm, min_ts, **kw):
    """Gradient of pixbw_step_loss w.r.t. [MLP params | post-softplus bkgd] + loss terms."""
    names = [n for n, _, _ in onerf.layer_specs(rd)]
    leaves = []
    for n in names:
        leaves += [p[n + ".weight"], p[n + ".bias"]]
    for t in leaves:
        t.requires_grad_(True)
        t.grad = None
    bk = torch.nn.functional.softplus(bkgd_raw).detach().requires_grad_(True)
    total, Ld, Lt = pixbw_step_loss(p, bk, raw, it_sample_size, n_samples, prm, min_ts, **kw)
    total.backward()
    g = torch.cat([t.grad.reshape(-1) for t in leaves] + [bk.grad.reshape(-1)])
    return g.detach(), (float(Ld.detach()), float(Lt.detach()), float(total.detach()))
