"""DeblurENeRF.training_step (the reference's operator API, models/deblur_e_nerf.py) on the HIP
path against the reference's own training_step run on the same reference-shaped batch
(tests/golden/step_*.npz: make_golden.gen_step binds the reference's training-path methods to
its own components, with nerfacc / RoMa restated by oracle/).  Needs an MI355X (marked gpu).

Checked against the reference's own float64 run of the same step (make_golden.gen_step "f64": the
module and batch in f64 on the f32 run's occupancy grid and samples) at max(1e-4, 4 x noise): the
north-star 1e-4 where the reference's f32 arithmetic is that accurate, else its own f32 rounding
noise -- the largest gap to the f64 run among the reference's f32 runs of the same step (as
configured and with the events reordered, ``*_f32p<k>``; the render background's gradient is a sum
of cancelling terms, 1e-1 .. 1e-2 f32-vs-f64 in the reference itself); see _check_f64.  The next
dynamic batch size to +-1.  The refractory-period gradient is the reference's full gradient
(``dtau_orig``): almost all of it flows through the camera pose (render timestamps ->
LinearTrajectory -> pixel rays -> sample positions / view directions, den_*_ray_grad and the
trajectory / pixel-ray backward kernels), ~1.5e-13 against ~1e-19..1e-25 without the pose path
(``dtau_orig_nopose``, kept in the fixture).
"""
import os
import re
import tempfile

import numpy as np
import pytest
import torch

from _util import flat_from_params, norm_rel
from oracle import nerf as onerf
from test_nerfacc_gpu import ARCH, _Draws
from test_ngp_gpu import _check_grid

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ngp_arch(z):
    import json
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    return ED(pos_encoding=json.loads(str(z["pos_encoding"])), dir_encoding=ED(degree=4),
              mlp_base=ED(hidden_activation="softplus", density_activation="shifted_trunc_exp", n_neurons=64,
                          n_hidden_layers=1, geo_feat_dim=15, weight_norm=False),
              mlp_head=ED(hidden_activation="softplus", radiance_activation="softplus", n_neurons=64,
                          n_hidden_layers=2, weight_norm=False))


def _fx(z, key, default):
    return z[key].item() if key in z.files else default


def build_model(z, mode="f32", sampler="occupancy", correction=None, eval_save=False, return_dir=False):
    """DeblurENeRF with the fixture's configuration (make_golden.gen_step: the chair-like defaults,
    or a step config's arch / contraction / aabb / near / far / cone / TV weight / learnable pixel
    bandwidth, e.g. configs[3]'s composition in step_ziggy_rd1.npz).  A fixture holding evaluation
    views (``file:`` entries, make_golden.gen_eval_epoch) has them written into the dataset
    directory first, so the constructor loads them (deblur_e_nerf.py:96-162)."""
    from deblur_e_nerf.models.deblur_e_nerf import DeblurENeRF
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    d = tempfile.mkdtemp(prefix="den_step_")
    cal = {k[4:]: z[k] for k in z.files if k.startswith("cal:")}
    poses = {k[5:]: z[k] for k in z.files if k.startswith("pose:")}
    np.savez(os.path.join(d, "camera_calibration.npz"), **cal)
    np.savez(os.path.join(d, "camera_poses.npz"), **poses)
    torch.save(torch.tensor(1_000_000), os.path.join(d, "max_refractory_period.pt"))
    for k in z.files:
        if k.startswith("file:"):
            path = os.path.join(d, k[len("file:"):])
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "wb") as f:
                f.write(z[k].tobytes())
    rd, S = int(z["rd"]), int(z["S"])
    aabb = [float(v) for v in z["aabb"]] if "aabb" in z.files else [-1.5, -1.5, -1.5, 1.5, 1.5, 1.5]
    nerf_cfg = ED(aabb=aabb, contraction_type=str(z["contraction"]) if "contraction" in z.files else "aabb",
                  occ_grid=ED(resolution=int(z["res"]), occ_thre=0.01, ema_decay=0.95, warmup_steps=256, n=16),
                  near_plane=float(_fx(z, "near", 1.43)), far_plane=float(_fx(z, "far", 6.63)),
                  render_step_size="auto", cone_angle=float(_fx(z, "cone", 0.0)), early_stop_eps=1e-4,
                  alpha_thre=0.0, test_chunk_size=16384, arch="mlp", mlp=ED(ARCH), load_state_dict=False,
                  freeze=False, compute_mode=mode, sampler=sampler)
    arch = str(z["arch"]) if "arch" in z.files else "mlp"
    if arch == "ngp":
        nerf_cfg.arch, nerf_cfg.ngp = "ngp", _ngp_arch(z)
    pixbw_free = bool(_fx(z, "pixbw_free", False))
    pb_names = ("tau_mil_it_eff_prod", "A_amp_inv", "A_loop_inv", "tau_out", "tau_sf", "tau_diff")
    m = DeblurENeRF(
        "test", ["novel_view"], 1, [0], 0.001, eval_save, None,
        ED(parameterize_mean_ct=True, load_state_dict=False,
           freeze=ED(p2n_contrast_threshold_ratio=False, mean_contrast_threshold=False, default=False)),
        ED(load_state_dict=False, freeze=False),
        ED(enable=bool(z["pixbw"]), it_sample_size=S, f_c_dominant_min=21, target_cumprob=ED(max_sample_lifetime=0.95),
           load_state_dict=False, freeze=ED(default=not pixbw_free, **{n: not pixbw_free for n in pb_names})),
        nerf_cfg, correction if correction is not None else ED(per_channel_log_it_scale=False, black_level_offset=True),
        ED(weight=ED(log_intensity_diff=1.0, log_intensity_tv=float(_fx(z, "tv", 1e-3)), nerf_mlp_weight_decay=1e-6),
           error_fn=ED(log_intensity_diff="huber", log_intensity_tv="l1"),
           normalize=ED(log_intensity_diff=True, log_intensity_tv=True)),
        ED(lpips_net="alex"),
        ED(algo="adam", lr=ED(default=1e-3, contrast_threshold=ED(p2n_contrast_threshold_ratio=1e-4,
                                                                 mean_contrast_threshold=1e-4),
                              pixel_bandwidth=ED({n: 1e-2 for n in pb_names} if pixbw_free else {})),
           relative_lr=ED(refractory_period=1e-3)),
        ED(algo="multi_step_lr", multi_step_lr=ED(milestones=[10], gamma=0.3), interval="epoch"),
        d, True, 131072)
    if arch == "ngp":
        rf = m.nerf.radiance_field
        p = {k[len("param:"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param:")}
        p["mlp_base.0.params"] = torch.from_numpy(z["table"])
        # the fixture holds the field parameters the reference rendered with (density shift included)
        rf.load_state_dict(dict(p, aabb=rf.aabb), strict=True)
        return m.to(DEV)
    p = onerf.build_params(rd, int(z["seed"]))
    m.nerf.radiance_field.flat_params.copy_(flat_from_params(p, rd))
    m = m.to(DEV)
    with torch.no_grad():
        m.nerf.radiance_field.mlp.sigma_layer.output_layer.bias.add_(float(z["sigma_bias_shift"]))
        if "rgb_weight_scale" in z.files:
            m.nerf.radiance_field.mlp.rgb_layer.output_layer.weight.mul_(float(z["rgb_weight_scale"]))
    return (m, d) if return_dir else m


def _rel(a, b):
    a = torch.as_tensor(np.asarray(a, np.float64) if not torch.is_tensor(a) else a.detach().cpu().double())
    b = torch.as_tensor(np.asarray(b, np.float64) if not torch.is_tensor(b) else b.detach().cpu().double())
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


EPS32 = 2.0 ** -24  # f32 unit roundoff
BOUND_MAX = 0.1  # the loosest bound a hot-path quantity may get without a well-conditioned companion check


def _check_vs(label, got, ref64, runs, base=1e-4, cond=None, companion=None):
    """|got - ref64| / |ref64| <= max(base, 4 x noise, 4 x cond u), noise = the largest gap of the
    reference's own f32 runs to its f64 run.  A bound above BOUND_MAX (the reference's f32 result
    itself unreliable) is accepted only beside a named ``companion`` check that pins the same
    quantity where it is well conditioned."""
    gaps = [_rel(r, ref64) for r in runs]
    noise = max(gaps)
    e = _rel(got, ref64)
    cfloor = EPS32 * cond if cond is not None else 0.0
    bound = max(base, 4.0 * noise, 4.0 * cfloor)
    extra = f", cond {cond:.3g} u {cfloor:.2e}" if cond is not None else ""
    print(f"  {label}: err vs f64 {e:.2e} (reference f32 runs {' '.join(f'{g:.1e}' for g in gaps)}{extra}, "
          f"bound {bound:.2e}{'; pinned by ' + companion if bound > BOUND_MAX else ''})")
    assert e <= bound, (label, e, bound)
    assert bound <= BOUND_MAX or companion, (label, "bound", bound, "with no well-conditioned companion check")
    return e


def _check_f64(z, key, got, base=1e-4, label=None, cond=None, mask=None, companion=None):
    """|got - ref_f64| / |ref_f64| <= max(base, 4 x noise): the north-star 1e-4 where the reference's
    f32 arithmetic is that accurate, else its own f32 rounding noise -- the largest gap to its f64
    run among its f32 runs of the same step: as configured, and with the events in N_PERM other
    orders (``<key>_f32p<k>``: every sum runs in another order, the f64 result is the same;
    make_golden.gen_step) -- or ``cond`` f32 roundoffs where the caller knows the quantity's
    condition number.  ``mask``: compare only those elements (all runs alike)."""
    sel = (lambda a: np.asarray(a.detach().cpu().double() if torch.is_tensor(a) else a)[mask]) if mask is not None \
        else (lambda a: a)
    runs = [z[key]] + [z[k] for k in sorted(z.files) if k.startswith(key + "_f32p")]
    return _check_vs(label or key, sel(got), sel(z[key + "_f64"]), [sel(r) for r in runs], base, cond, companion)


def _tv_mask(z, n_events):
    """Events whose TV difference d = log I(subdiff end) - log I(subdiff start) (the reference's
    f64 run) is resolved in f32: |d| > 16 x the f32 error of d -- the reference's own f32 run's
    error on that event, or the median over events if larger (renders in f32 are ~1e-6 off in
    log I).  There the L1 term's sign, hence its gradient, is defined by the reference's
    arithmetic; below it (rays that see nearly the same intensity at both timestamps) the sign is
    f32 noise in the reference itself (its f32 runs are 30-55 % off its f64 run on these groups)."""
    a, b = z["li_g2_f64"].reshape(-1, n_events), z["li_g3_f64"].reshape(-1, n_events)
    a32 = z["li_g2"].reshape(-1, n_events).astype(np.float64)
    b32 = z["li_g3"].reshape(-1, n_events).astype(np.float64)
    d = b - a
    err = np.abs((b32 - a32) - d)
    noise = np.maximum(err, np.median(err))
    return (np.abs(d) > 16.0 * noise).all(axis=0)


class _BkgdTap:
    """Per NeRF.forward call: d loss / d colour x (1 - opacity) per ray (what the render
    background's gradient sums, C = C_fg + bkgd (1 - O)), recorded as make_golden records the
    reference's (``bkray_<call>``)."""

    def __init__(self, m):
        self.rows = []
        orig = m.nerf.forward

        def fwd(o, d):
            rad, op, dp, mspr = orig(o, d)
            slot = len(self.rows)
            self.rows.append(None)
            keep = (1 - op.detach()).clone()
            rad = _GradTap.apply(rad, lambda g, i=slot, w=keep: self.rows.__setitem__(
                i, (g.detach() * (w[..., None] if g.dim() > w.dim() else w)).double().cpu().reshape(-1)))
            return rad, op, dp, mspr
        m.nerf.forward = fwd


def _check_bkgd(z, m, bk, n_events):
    """The render background's gradient: its sum over rays cancels (the reference's own f32 runs are
    1e-2..1 off its f64 run), so each ray's term is checked before the sum -- all rays of the diff
    groups, the TV groups' rays of well-conditioned events (_tv_mask)."""
    calls = sorted(int(k[6:]) for k in z.files if re.fullmatch(r"bkray_\d+", k))
    ours = torch.cat(bk.rows).numpy()
    ref32 = np.concatenate([z[f"bkray_{c}"].reshape(-1) for c in calls])
    ref64 = np.concatenate([z[f"bkray_{c}_f64"].reshape(-1) for c in calls])
    assert ours.shape == ref64.shape, (ours.shape, ref64.shape)
    tvm = _tv_mask(z, n_events)
    per_call = ref64.size // len(calls)
    keep = np.ones(ref64.size, bool)
    for gi in (2, 3):  # calls in group order: diff start, diff end, tv start, tv end
        idx = np.arange(gi * per_call, (gi + 1) * per_call)
        keep[idx] = tvm[idx % n_events]
    _check_vs(f"background gradient per ray ({int(keep.sum())} of {keep.size} rays)", ours[keep], ref64[keep],
              [ref32[keep]])
    _check_f64(z, "grad_bkgd_orig", m.nerf.parametrizations.render_bkgd.original.grad,
               companion="the per-ray terms above")


class _GradTap(torch.autograd.Function):
    """Identity whose backward hands the incoming gradient to ``fn`` (make_golden's recorder)."""

    @staticmethod
    def forward(ctx, x, fn):
        ctx.fn = fn
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.fn(g)
        return g, None


class _TsHook:
    """d loss / d timestamp through every render_log_intensity call (trajectory -> rays -> render,
    the pose path's input), recorded by an identity in front of the call as make_golden records
    the reference's (dts_g*); also the gradient of the loss's normalising constant (the mean
    contrast threshold passed to Loss.compute), the term the mean-C gradient cancels against."""

    def __init__(self, m):
        self.grads, orig = [], m.render_log_intensity
        self.g_c = []
        self.bk = _BkgdTap(m)

        def rli(timestamp, *a, **k):
            if timestamp.requires_grad:
                slot = len(self.grads)
                self.grads.append(None)
                timestamp = _GradTap.apply(timestamp,
                                           lambda g, i=slot: self.grads.__setitem__(i, g.detach().cpu().clone()))
            return orig(timestamp, *a, **k)
        m.render_log_intensity = rli
        comp = m.loss.compute

        def compute(ev, diff, sub, c):
            c = _GradTap.apply(c, lambda g: self.g_c.append(float(g.detach().sum())))
            return comp(ev, diff, sub, c)
        m.loss.compute = compute

    def per_group(self):
        out = []
        for g in self.grads:
            out.extend(list(g) if g.dim() == 2 else [g])  # pixel bandwidth off: one (4, N) call
        return out


def _replay_randint(z, monkeypatch):
    """The reference's torch.randint draws of its occupancy update (the cone branch's random camera
    per cell point, nerf.py:178-181; make_golden records them as occ_randint_<k>), replayed in order
    through models/nerf._randint."""
    from deblur_e_nerf.models import nerf as nerf_lib
    keys = sorted((k for k in z.files if k.startswith("occ_randint_")), key=lambda k: int(k.rsplit("_", 1)[1]))
    draws = [torch.from_numpy(z[k]) for k in keys]
    cone = float(_fx(z, "cone", 0.0))
    assert (len(draws) > 0) == (cone > 0), (cone, keys)

    def replay(high, size, device=None):
        r = draws.pop(0)
        assert tuple(r.shape) == tuple(size) and int(r.max()) < high
        return r.to(device)
    monkeypatch.setattr(nerf_lib, "_randint", replay)


def _batch(z):
    ev = {k[6:]: torch.from_numpy(z[k]).to(DEV) for k in z.files if k.startswith("event:")}
    nz = {k[11:]: torch.from_numpy(z[k]).to(DEV) for k in z.files if k.startswith("normalized:")}
    return {"event": ev, "normalized": nz}


def _check_common(z, m, hook, fixture):
    """Loss, next batch size, C+/C- ratio, mean C, background, tau_r and the per-call timestamp
    gradients, each against the reference's f64 run with the f32 run's gap as the floor."""
    ctp = m.contrast_threshold.parametrizations
    _check_f64(z, "d_p2n_orig", ctp.p2n_contrast_threshold_ratio.original.grad)
    # dL/dC_mean = (the C+/C- path through the measured log-intensity change) + (the normalising
    # constant's path): two terms ~1e4 x their sum on these batches, so |dL/dc| rounded to f32 is
    # the floor (the reference's own f32 run is 1.7e-3 off on step_nopixbw_rd1)
    orig = ctp.mean_contrast_threshold.original
    with torch.enable_grad():
        fprime = float(torch.autograd.grad(m.contrast_threshold.mean_contrast_threshold.sum(), orig)[0])
    d_mean = abs(float(z["d_mean_ct_orig_f64"])) / abs(fprime)
    _check_f64(z, "d_mean_ct_orig", orig.grad, cond=abs(sum(hook.g_c)) / d_mean)
    n_events = int(z["event:end_ts"].size)
    _check_bkgd(z, m, hook.bk, n_events)
    dtau = m.refractory_period.parametrizations._refractory_period.original.grad
    # tau_r's gradient: the reference's full gradient, almost all of it through the camera pose, at
    # the north-star 1e-4 relative or 4 x the reference f32 run's own error (no per-term floor: a
    # zero or pose-free gradient fails)
    ref64 = float(z["dtau_orig_f64"])
    e_tau = abs(float(dtau) - ref64)
    runs = [float(z["dtau_orig"])] + [float(z[k]) for k in z.files if k.startswith("dtau_orig_f32p")]
    b_tau = max(1e-4 * abs(ref64), 4.0 * max(abs(r - ref64) for r in runs))
    print(f"  dtau: |err| {e_tau:.3e} ({e_tau / abs(ref64):.2e} relative) vs bound {b_tau:.3e} (|dtau| {abs(ref64):.3e}, "
          f"{abs(float(z['dtau_orig_nopose'])):.1e} without the pose path)")
    assert e_tau <= b_tau
    groups = hook.per_group()
    ref = [k for k in z.files if re.fullmatch(r"dts_g\d+", k)]
    assert len(groups) == len(ref) == 4, (len(groups), ref)
    tvm = _tv_mask(z, n_events)
    for i, g in enumerate(groups):
        if i < 2:
            _check_f64(z, f"dts_g{i}", g, label=f"d loss / d render ts, group {i}")
            continue
        # the TV groups: an L1 of differences, sign-defined only where the difference is resolved
        _check_f64(z, f"dts_g{i}", g, mask=tvm,
                   label=f"d loss / d render ts, group {i}, {int(tvm.sum())} of {n_events} events resolved")
        _check_f64(z, f"dts_g{i}", g, label=f"d loss / d render ts, group {i}, all events",
                   companion="the resolved events")
    pb = [k for k in z.files if k.startswith("dpixbw:") and not k.endswith("_f64") and "_f32p" not in k]
    for k in pb:
        name = k[len("dpixbw:"):]
        # pinned per parameter against the reference's f64 pixel-bandwidth backward at 1e-4 on
        # well-conditioned inputs: tests/test_pixbw_gpu.py::test_pixel_bandwidth_matches_reference_golden (each parameter at 1e-4)
        _check_f64(z, k, getattr(m.pixel_bandwidth.parametrizations, name).original.grad,
                   companion="tests/test_pixbw_gpu.py (parameter gradients vs the reference's f64 run)")
    print(f"[{fixture}] dtau {float(dtau):.6e} vs the reference {float(z['dtau_orig']):.6e} "
          f"(f64 {float(z['dtau_orig_f64']):.6e}; {float(z['dtau_orig_nopose']):.2e} without the pose path)")


@pytest.mark.parametrize("fixture", ["step_nopixbw_rd1", "step_pixbw_rd1"])
def test_training_step_matches_reference(golden_dir, fixture, monkeypatch):
    from deblur_e_nerf.external import marching
    z = np.load(os.path.join(golden_dir, fixture + ".npz"))
    m = build_model(z)
    m.train()
    hook = _TsHook(m)
    jit = [z[f"jitter_{i}"] for i in range(4)]
    draws = [z["occ_u"]] + (jit if bool(z["pixbw"]) else [np.concatenate(jit)])
    monkeypatch.setattr(marching, "_uniform", _Draws(draws))
    _replay_randint(z, monkeypatch)
    loss = m.training_step(_batch(z), 0)
    loss.backward()
    torch.cuda.synchronize()
    print(f"[{fixture}] loss {float(loss):.7f} vs {float(z['loss']):.7f}; batch size {m.train_batch_size} vs "
          f"{int(z['new_batch_size'])}")
    _check_grid(m.nerf.occupancy_grid, z)
    _check_f64(z, "loss", loss)
    assert abs(m.train_batch_size - int(z["new_batch_size"])) <= 1
    flat = torch.cat([p.grad.detach().reshape(-1) for _, p in m.nerf.radiance_field.mlp.named_parameters()]).cpu()
    _check_f64(z, "grad_pick", flat[torch.from_numpy(z["grad_pick_idx"])], label="MLP gradient (4096 picks)")
    _check_f64(z, "grad_norm", flat.double().norm(), label="MLP gradient norm")
    _check_common(z, m, hook, fixture)


@pytest.mark.parametrize("fixture", ["step_ngp_nopixbw_rd1", "step_ziggy_rd1"])
def test_training_step_ngp_matches_reference(golden_dir, fixture, monkeypatch):
    """The same with nerf.arch = ngp (the configs' default field): the reference training_step
    with its NGPradianceField (tcnn.Encoding restated by oracle/tcnn.py), F32 kernels here.
    step_ziggy_rd1 is configs[3]'s model composition (07_ziggy_and_fuzz_hdr.yaml): unbounded-sphere
    contraction, cone marching, pixel bandwidth S = 30 with learnable sensor parameters, TV 0.1.
    Every field gradient (hash table included) tensor-wise against the f64 run."""
    from deblur_e_nerf.external import marching
    z = np.load(os.path.join(golden_dir, fixture + ".npz"))
    m = build_model(z)
    m.train()
    hook = _TsHook(m)
    jit = [z[f"jitter_{i}"] for i in range(4)]
    draws = [z["occ_u"]] + (jit if bool(z["pixbw"]) else [np.concatenate(jit)])
    monkeypatch.setattr(marching, "_uniform", _Draws(draws))
    _replay_randint(z, monkeypatch)
    loss = m.training_step(_batch(z), 0)
    loss.backward()
    torch.cuda.synchronize()
    print(f"[{fixture}] loss {float(loss):.7f} vs {float(z['loss']):.7f}; batch size {m.train_batch_size} vs "
          f"{int(z['new_batch_size'])}")
    _check_grid(m.nerf.occupancy_grid, z)
    _check_f64(z, "loss", loss)
    assert abs(m.train_batch_size - int(z["new_batch_size"])) <= 1
    for k, p in m.nerf.radiance_field.named_parameters():
        _check_f64(z, f"grad:{k}", p.grad)
    _check_common(z, m, hook, fixture)


def test_configure_optimizers_and_fit_step(golden_dir, monkeypatch):
    """configure_optimizers (den Adam per parameter group, MultiStepLR) and one fit_step."""
    from deblur_e_nerf.external import marching
    z = np.load(os.path.join(golden_dir, "step_nopixbw_rd1.npz"))
    m = build_model(z)
    m.train()
    opt = m.configure_optimizers()["optimizer"]
    before = m.nerf.radiance_field.flat_params.clone()
    jit = np.concatenate([z[f"jitter_{i}"] for i in range(4)])
    monkeypatch.setattr(marching, "_uniform", _Draws([z["occ_u"], jit]))
    loss = m.fit_step(_batch(z), 0, opt)
    torch.cuda.synchronize()
    step = (m.nerf.radiance_field.flat_params - before).abs()
    assert torch.isfinite(loss) and float(step.max()) > 0
    # Adam's first step moves every parameter with a non-zero gradient by ~lr
    assert float(step.max()) <= 1.01e-3


def _event_batch(N, seed, img=800, ts_lo=1.5e8, ts_hi=9.5e8):
    """A reference-shaped batch (datamodule.py:215-247) of N events, as tests/golden/make_golden.py
    builds them: events (1, N, ...) and the normalized samples (1, N)."""
    g = torch.Generator().manual_seed(seed)
    num_pos = (torch.rand(N, generator=g) < 0.5).long()
    end_ts = (torch.rand(N, generator=g, dtype=torch.float64) * (ts_hi - ts_lo) + ts_lo).long()
    start_ts = end_ts - (-torch.log(torch.rand(N, generator=g, dtype=torch.float64)) * 2e6 + 2e4).long()
    position = torch.rand(N, 2, generator=g) * (img - 1)
    u = torch.rand(3, N, generator=g, dtype=torch.float64)
    ev = dict(position=position[None], start_ts=start_ts[None], end_ts=end_ts[None], num_pos=num_pos[None],
              num_neg=(1 - num_pos)[None])
    nz = dict(ts_diff=torch.ones(1, N, dtype=torch.float64), diff_start_ts=u[0][None],
              ts_subdiff=(1 - torch.sqrt(1 - u[1]))[None], subdiff_start_ts=u[2][None])
    return dict(event=ev, normalized=nz)


def _slice(batch, a, b):
    return {grp: {k: v[:, a:b].contiguous().to(DEV) for k, v in d.items()} for grp, d in batch.items()}


def test_gradient_accumulation_equals_one_big_batch(golden_dir, monkeypatch):
    """PL accumulate_grad_batches semantics (configs[3]: 07_ziggy_and_fuzz_hdr.yaml:203,
    accumulate_grad_batches 8; deblur_e_nerf.py:465 occupancy update on the first micro-batch only,
    :1286-1291 batch-size update on the second-to-last): 8 micro-batches of n events through
    fit_step (loss / 8 accumulated, one optimizer step on the last) give the gradient of ONE
    training_step on the 8n-event batch -- the same marching draws, split per micro-batch -- and
    leave the parameters untouched until the 8th.  F32 at the north-star 1e-4 (measured 2.7e-5: the
    loss gradient is a difference of nearby renders, so f32 summation order shows at ~1e-5)."""
    from deblur_e_nerf.external import marching
    z = np.load(os.path.join(golden_dir, "step_nopixbw_rd1.npz"))
    n, acc = 40, 8
    big = _event_batch(n * acc, seed=31)
    jit = torch.rand(4, n * acc, generator=torch.Generator().manual_seed(32))
    occ_u = z["occ_u"]

    m_big = build_model(z)
    m_big.train()
    monkeypatch.setattr(marching, "_uniform", _Draws([occ_u, jit.reshape(-1).numpy()]))
    loss_big = m_big.training_step(_slice(big, 0, n * acc), 0)
    loss_big.backward()
    g_big = torch.cat([p.grad.detach().reshape(-1) for p in m_big.parameters() if p.grad is not None]).cpu()

    m_acc = build_model(z)
    m_acc.train()
    m_acc.trainer.accumulate_grad_batches = acc
    opt = m_acc.configure_optimizers()["optimizer"]
    before = m_acc.nerf.radiance_field.flat_params.detach().clone()
    g_acc = None
    for k in range(acc):
        draws = ([occ_u] if k == 0 else []) + [jit[:, k * n:(k + 1) * n].reshape(-1).numpy()]
        monkeypatch.setattr(marching, "_uniform", _Draws(draws))
        if k == acc - 1:
            # fit_step's last micro-batch, spelled out to read the accumulated gradient before
            # the optimizer step consumes it
            loss = m_acc.training_step(_slice(big, k * n, (k + 1) * n), k)
            (loss / acc).backward()
            g_acc = torch.cat([p.grad.detach().reshape(-1) for p in m_acc.parameters()
                               if p.grad is not None]).cpu()
            opt.step()
            torch.cuda.synchronize()
            assert not torch.equal(m_acc.nerf.radiance_field.flat_params, before)
            break
        m_acc.fit_step(_slice(big, k * n, (k + 1) * n), k, opt)
        torch.cuda.synchronize()
        assert torch.equal(m_acc.nerf.radiance_field.flat_params, before)  # no step before the 8th
    e = norm_rel(g_acc, g_big)
    print(f"8 accumulated micro-batches vs one 8x batch: gradient rel err {e:.2e} "
          f"(loss {float(loss_big):.6f})")
    assert g_acc.shape == g_big.shape and e <= 1e-4
