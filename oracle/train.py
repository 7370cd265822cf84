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
