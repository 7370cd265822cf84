"""Generate golden fixtures by RUNNING the reference's own PyTorch modules.

Runs only in the build container (the reference tree is absent on the GPU box):

    python tests/golden/make_golden.py

Each fixture is a small ``.npz`` (inputs + the reference's outputs/gradients,
plain arrays, no pickles).  The reference modules are imported through
``_refload`` (namespace shim, import-only stand-ins for easydict/cv2/roma/nerfacc
enum/tinycudann).  What each fixture pins:

* ``mlp_rd{1,3}.npz``   -- external/mlp.py ``VanillaNeRFRadianceField`` forward +
                           backward (softplus(beta=100) hidden, shifted_trunc_exp
                           density (external/ngp.py:45-65), softplus radiance), f32
                           and f64 outputs, weights = PyTorch default Linear init
                           under ``torch.manual_seed(seed)`` (re-creatable anywhere).
* ``foh.npz``           -- utils/control.py ``foh_cont2discrete`` (efficient and
                           block-expm branches) on pixel-bandwidth-shaped systems.
* ``pixbw_S{16,30}.npz`` -- models/pixel_bandwidth.py ``PixelBandwidth.forward``:
                           the 4-call training sequence (reset on the first call,
                           deblur_e_nerf.py:472-526) with intensity samples given
                           as leaf tensors; outputs, module state and gradients.
* ``loss.npz``          -- loss_metric/loss.py ``Loss.compute`` (huber/l1,
                           normalized, masked means) + gradients.
* ``ct.npz``            -- models/event_generation_params.py ContrastThreshold
                           forward (counts -> delta log I).
* ``events.npz``        -- the event preparation of DeblurENeRF.training_step:
                           ContrastThreshold + RefractoryPeriod forward (modules
                           run as-is), then the diff / subdiff timestamp derivation
                           of deblur_e_nerf.py:418-455, executed from the reference
                           file's own text (located by its comment markers at
                           generation time; nothing of it is stored), for the three
                           loss-weight cases (both terms, diff only, TV only).
* ``rays.npz``          -- models/nerf.py NeRF.pixel_params_to_ray (pixel + pose ->
                           ray origin / unit direction), with and without the
                           leading render-group dimension.
* ``queue_*.npz``       -- data/datasets.py Event.queue_raw_events, colorize_events,
                           undistort_events (no distortion: the cast) and
                           extract_max_refractory_period, the reference's loops run on
                           synthetic raw_events.npz directories (repeated timestamps,
                           bursts, single-event pixels, unsorted input, hot pixels).
"""
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import _refload  # noqa: E402

# tinycudann is imported (not used) by external/ngp.py, which holds trunc_exp.
sys.modules.setdefault("tinycudann", types.ModuleType("tinycudann"))

# EDS-assumed DVS constants (reference scripts/eds_to_esim.py:68-79).
EDS = dict(
    input_time_const_eff_it_prod=(35e-12 * 25e-3) / 2000e-12,
    miller_time_const_eff_it_prod=(0.6e-12 * 25e-3) / 2000e-12,
    amplifier_gain=140.0,
    closed_loop_gain=1 / 0.7,
    output_time_const=25e-6,
    sf_cutoff_freq=16400.0,
    diff_amp_cutoff_freq=82000.0,
)
# A second, perturbed sensor (slower pixel) to exercise other stiffness regimes.
PERTURBED = dict(
    input_time_const_eff_it_prod=2.0e-3,
    miller_time_const_eff_it_prod=3.0e-5,
    amplifier_gain=60.0,
    closed_loop_gain=1.6,
    output_time_const=80e-6,
    sf_cutoff_freq=3000.0,
    diff_amp_cutoff_freq=9000.0,
)
CT = dict(pos_contrast_threshold=0.25, neg_contrast_threshold=0.2)


def _calib_dir(consts):
    d = tempfile.mkdtemp(prefix="den_calib_")
    arrs = {k: np.array(v, dtype=np.float32) for k, v in consts.items()}
    for k, v in CT.items():
        arrs[k] = np.array(v, dtype=np.float32)
    arrs["refractory_period"] = np.array(0)
    arrs["bayer_pattern"] = np.array("")
    np.savez(os.path.join(d, "camera_calibration.npz"), **arrs)
    return d


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


# ----------------------------------------------------------------------------
def gen_mlp(rd, seed, contraction="aabb", density="shifted_trunc_exp"):
    """VanillaNeRFRadianceField forward/backward; contraction "aabb" (mlp_rd{rd}.npz) or the
    unbounded "sphere" / "tanh" input-space contractions (mlp_rd{rd}_{contraction}.npz: mlp.py:321-335,
    ngp.py:68-106), whose positions reach 4x the box so the contracted shells are exercised."""
    mlp = _refload.load("external.mlp")
    ngp = _refload.load("external.ngp")
    nerfm = _refload.load("models.nerf")
    ContractionType = sys.modules["nerfacc"].ContractionType
    ctype = {"aabb": ContractionType.AABB, "sphere": ContractionType.UN_BOUNDED_SPHERE,
             "tanh": ContractionType.UN_BOUNDED_TANH}[contraction]
    torch.manual_seed(seed)
    field = mlp.VanillaNeRFRadianceField(
        aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], net_depth=8, net_width=256,
        skip_layer=4, net_depth_condition=1, net_width_condition=128, num_dim=3,
        contraction_type=ctype, radiance_dim=rd,
        hidden_activation=torch.nn.Softplus(beta=100),
        density_activation=nerfm.NeRF.DENSITY_ACTIVATION_NAME_TO_FN[density],
        radiance_activation=torch.nn.Softplus(beta=1),
        pos_encoder_max_deg=10, view_encoder_max_deg=4, weight_norm=False)
    g = torch.Generator().manual_seed(1000 + seed)
    n = 512
    # positions: mostly inside the AABB, some outside (selector = 0); unbounded contractions: up to
    # 4x the box, the sphere's |x| > 1 shell and the tanh tails
    span = 1.8 if contraction == "aabb" else 6.0
    x = (torch.rand(n, 3, generator=g) * 2 * span - span).float()
    d = torch.randn(n, 3, generator=g)
    d = d / d.norm(dim=-1, keepdim=True)
    g_rgb = torch.randn(n, rd, generator=g)
    g_sig = torch.randn(n, 1, generator=g)
    names = [k for k, _ in field.named_parameters()]
    out = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        f = field.to(dt)
        f.zero_grad()
        rgb, sig = f(x.to(dt), d.to(dt))
        (rgb * g_rgb.to(dt)).sum().add_((sig * g_sig.to(dt)).sum()).backward()
        out[f"rgb_{tag}"] = rgb.detach().numpy()
        out[f"sigma_{tag}"] = sig.detach().numpy()
        for k, p in f.named_parameters():
            gr = p.grad.detach().numpy()
            out[f"gnorm_{tag}:{k}"] = np.array(np.linalg.norm(gr.astype(np.float64)))
            out[f"gsum_{tag}:{k}"] = np.array(gr.astype(np.float64).sum())
            if tag == "f32" and (p.numel() <= 40000 or k.endswith("hidden_layers.0.weight")):
                out[f"grad:{k}"] = gr
    field.float()
    wsum = {f"wsum:{k}": np.array(p.detach().double().sum().item()) for k, p in field.named_parameters()}
    name = f"mlp_rd{rd}.npz" if contraction == "aabb" else f"mlp_rd{rd}_{contraction}.npz"
    if density != "shifted_trunc_exp":
        name = name.replace(".npz", f"_{density}.npz")
    save(name, seed=seed, contraction=np.array(contraction), density=np.array(density), x=x.numpy(), d=d.numpy(),
         g_rgb=g_rgb.numpy(), g_sigma=g_sig.numpy(), param_names=np.array(names), **out, **wsum)


# ----------------------------------------------------------------------------
def gen_foh():
    control = _refload.load("utils.control")
    g = torch.Generator().manual_seed(3)
    B = 64
    res = {}
    A = torch.zeros(B, 4, 4, dtype=torch.float64)
    two_zeta_w = 10 ** (torch.rand(B, generator=g, dtype=torch.float64) * 3 + 3)
    w2 = 10 ** (torch.rand(B, generator=g, dtype=torch.float64) * 5 + 6)
    wsf = 10 ** (torch.rand(B, generator=g, dtype=torch.float64) * 2 + 3)
    wdf = 10 ** (torch.rand(B, generator=g, dtype=torch.float64) * 2 + 4)
    A[:, 0, 0] = -two_zeta_w
    A[:, 0, 1] = -w2
    A[:, 1, 0] = 1
    A[:, 2, 1] = wsf
    A[:, 2, 2] = -wsf
    A[:, 3, 2] = wdf
    A[:, 3, 3] = -wdf
    Bm = torch.zeros(B, 4, 1, dtype=torch.float64)
    Bm[:, 0, 0] = w2
    C = torch.tensor([[0, 0, 1, 0], [0, 0, 0, 1]], dtype=torch.float64).expand(B, 2, 4)
    D = torch.zeros(B, 2, 1, dtype=torch.float64)
    dt = 10 ** (torch.rand(B, generator=g, dtype=torch.float64) * 4 - 7)
    res.update(A=A.numpy(), B=Bm.numpy(), dt=dt.numpy())
    for dtype, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        sys_ = control.StateSpace(A=A.to(dtype), B=Bm.to(dtype), C=C.to(dtype), D=D.to(dtype))
        for eff in (True, False):
            sd = control.foh_cont2discrete(sys_, dt.to(dtype), is_state_preserved=True, is_efficient=eff)
            t = f"{tag}_{'eff' if eff else 'blk'}"
            res[f"Ad_{t}"] = sd.A.numpy()
            res[f"Bd_{t}"] = sd.B.numpy()
            res[f"Btd_{t}"] = sd.B_tilde.numpy()
    save("foh.npz", **res)


# ----------------------------------------------------------------------------
def _intensity_of(ts_ns, base, amp, freq, phase):
    # smooth positive intensity trace per event (ts in ns, f64)
    t = ts_ns * 1e-9
    return base * torch.exp(amp * torch.sin(2 * np.pi * freq * t + phase))


def gen_pixbw(S, consts, tag):
    pbm = _refload.load("models.pixel_bandwidth")
    ED = sys.modules["easydict"].EasyDict
    calib = _calib_dir(consts)
    min_ts = torch.tensor(100_000_000, dtype=torch.int64)  # 0.1 s
    pb = pbm.PixelBandwidth(calib, min_ts, 21, ED(max_sample_lifetime=0.95))
    g = torch.Generator().manual_seed(11 + S)
    N = 96
    base = 10 ** (torch.rand(N, generator=g, dtype=torch.float64) * 3 - 2)  # 0.01 .. 10
    amp = torch.rand(N, generator=g, dtype=torch.float64) * 1.5
    freq = 10 ** (torch.rand(N, generator=g, dtype=torch.float64) * 3)      # 1..1000 Hz
    phase = torch.rand(N, generator=g, dtype=torch.float64) * 6.28
    # event interval [start, end] in ns (f64 start after refractory, i64 end)
    end_ts = (torch.rand(N, generator=g, dtype=torch.float64) * 0.8e9 + 0.15e9).floor()
    interval = -torch.log(torch.rand(N, generator=g, dtype=torch.float64)) * 1e6 + 2e3
    start_ts = end_ts - interval
    # the four render timestamps of one training step (deblur_e_nerf.py:419-455)
    sub_w = torch.rand(N, generator=g, dtype=torch.float64)
    sub_len = (end_ts - start_ts) * torch.rand(N, generator=g, dtype=torch.float64) ** 2
    sub_start = torch.lerp(start_ts, torch.maximum(end_ts - sub_len, start_ts), sub_w)
    sub_end = torch.minimum(sub_start + sub_len, end_ts)
    call_ts = [start_ts, end_ts, sub_start, sub_end]
    gens = [torch.full((S - 1, N), 0.5, dtype=torch.float64),
            torch.rand(S - 1, N, generator=g, dtype=torch.float64)]
    coef = torch.randn(4, N, generator=g, dtype=torch.float64)

    out = dict(S=S, N=N, min_ts=min_ts.numpy(), base=base.numpy(), amp=amp.numpy(),
               freq=freq.numpy(), phase=phase.numpy(), coef=coef.numpy(),
               call_ts=torch.stack(call_ts).numpy(), gen_dirac=gens[0].numpy(),
               gen_unif=gens[1].numpy(),
               **{f"calib:{k}": np.array(v, dtype=np.float32) for k, v in consts.items()})
    pnames = ["tau_mil_it_eff_prod", "A_amp_inv", "A_loop_inv", "tau_out", "tau_sf", "tau_diff"]
    for gi, gen in enumerate(gens):
        for dtype, dtag in ((torch.float32, "f32"), (torch.float64, "f64")):
            pb.zero_grad()
            pbd = pb.to(dtype) if dtype == torch.float64 else pb.float()
            leaves = []

            def fn(ts):
                it = _intensity_of(ts, base, amp, freq, phase).to(dtype)
                it = it.detach().requires_grad_(True)
                leaves.append(it)
                return (it, torch.tensor(0.0), 128.0, torch.ones_like(it, dtype=torch.bool))

            outs = []
            for c in range(4):
                y, aux = pbd(gen, call_ts[c], fn, reset_diff=(c == 0))
                outs.append(y)
                if c == 0:
                    out[f"delta_g{gi}_{dtag}"] = pbd.reset_delta_log_it.detach().numpy()
            loss = sum((outs[c] * coef[c].to(dtype)).sum() for c in range(4))
            loss.backward()
            for c in range(4):
                out[f"logit_g{gi}_{dtag}_c{c}"] = outs[c].detach().numpy()
                out[f"it_g{gi}_{dtag}_c{c}"] = leaves[c].detach().numpy()
                out[f"dit_g{gi}_{dtag}_c{c}"] = leaves[c].grad.numpy()
            for pn in pnames:
                orig = getattr(pbd.parametrizations, pn).original
                out[f"dparam_g{gi}_{dtag}:{pn}"] = orig.grad.detach().numpy()
                out[f"param_{dtag}:{pn}"] = getattr(pbd, pn).detach().numpy()
                out[f"orig_{dtag}:{pn}"] = orig.detach().numpy()
    pb.float()
    save(f"pixbw_S{S}_{tag}.npz", **out)


# ----------------------------------------------------------------------------
def gen_loss():
    lossm = _refload.load("loss_metric.loss")
    ED = sys.modules["easydict"].EasyDict
    g = torch.Generator().manual_seed(5)
    N = 1000
    out = {}
    # ("mape", "l1") last: the earlier variants' draws are unchanged (the generator runs in order)
    for efn_diff, efn_tv in (("huber", "l1"), ("l1", "huber"), ("mse", "mse"), ("mape", "l1")):
        L = lossm.Loss(ED(log_intensity_diff=1.0, log_intensity_tv=1e-3),
                       ED(log_intensity_diff=efn_diff, log_intensity_tv=efn_tv),
                       ED(log_intensity_diff=True, log_intensity_tv=True))
        num_pos = (torch.rand(N, generator=g) < 0.5).long()
        num_neg = 1 - num_pos
        end_ts = (torch.rand(N, generator=g, dtype=torch.float64) * 1e9).floor().long() + 10**8
        start_ts = end_ts.double() - (torch.rand(N, generator=g, dtype=torch.float64) * 2e6 + 1e3)
        Cp, Cn = 0.25, 0.2
        lid = (num_pos * Cp - num_neg * Cn).float()
        ts_diff = (end_ts - start_ts) * 1.0
        d_lid = (torch.randn(N, generator=g) * 0.3).requires_grad_(True)
        s_lid = (torch.randn(N, generator=g) * 0.1).requires_grad_(True)
        d_valid = torch.rand(N, generator=g) < 0.9
        s_valid = torch.rand(N, generator=g) < 0.8
        mct = torch.tensor(0.225, requires_grad=True)
        be = ED(log_intensity_diff=lid, end_ts=end_ts, start_ts=start_ts)
        bd = ED(log_intensity_diff=d_lid, ts_diff=ts_diff, is_valid=d_valid)
        bs = ED(log_intensity_diff=s_lid, is_valid=s_valid)
        res = L.compute(be, bd, bs, mct)
        total = res.log_intensity_diff * 1.0 + res.log_intensity_tv * 1e-3
        total.backward()
        t = f"{efn_diff}_{efn_tv}"
        out.update({f"{t}:num_pos": num_pos.numpy(), f"{t}:end_ts": end_ts.numpy(),
                    f"{t}:start_ts": start_ts.numpy(), f"{t}:lid": lid.numpy(),
                    f"{t}:d_lid": d_lid.detach().numpy(), f"{t}:s_lid": s_lid.detach().numpy(),
                    f"{t}:d_valid": d_valid.numpy(), f"{t}:s_valid": s_valid.numpy(),
                    f"{t}:L_diff": res.log_intensity_diff.detach().numpy(),
                    f"{t}:L_tv": res.log_intensity_tv.detach().numpy(),
                    f"{t}:g_d_lid": d_lid.grad.numpy(), f"{t}:g_s_lid": s_lid.grad.numpy(),
                    f"{t}:g_mct": mct.grad.numpy()})
    out["Cp"] = np.array(0.25)
    out["Cn"] = np.array(0.2)
    save("loss.npz", **out)


def gen_ct():
    egp = _refload.load("models.event_generation_params")
    ED = sys.modules["easydict"].EasyDict
    calib = _calib_dir(EDS)
    ct = egp.ContrastThreshold(calib, parameterize_mean_ct=True)
    g = torch.Generator().manual_seed(9)
    N = 300
    num_pos = torch.randint(0, 3, (N,), generator=g)
    num_neg = torch.randint(0, 3, (N,), generator=g)
    o = ct(ED(num_pos=num_pos, num_neg=num_neg))
    save("ct.npz", num_pos=num_pos.numpy(), num_neg=num_neg.numpy(),
         lid=o.log_intensity_diff.detach().numpy(),
         pos_ct=ct.pos_contrast_threshold.detach().numpy(),
         neg_ct=ct.neg_contrast_threshold.detach().numpy(),
         mean_ct=ct.mean_contrast_threshold.detach().numpy())


def _training_step_ts_code():
    """The timestamp-derivation block of DeblurENeRF.training_step, read from the
    reference file (deblur_e_nerf.py:418-455) between its own comment markers."""
    src = open(os.path.join(_refload.REF_ROOT, "deblur_e_nerf/models/deblur_e_nerf.py")).read().splitlines()
    a = next(i for i, l in enumerate(src) if "# derive the ts. for log-intensity supervision" in l)
    b = next(i for i in range(a, len(src)) if src[i].strip() == "batch.subdiff = None")
    import textwrap
    return textwrap.dedent("\n".join(src[a:b + 1]))


def gen_events():
    egp = _refload.load("models.event_generation_params")
    ED = sys.modules["easydict"].EasyDict
    d = _calib_dir(EDS)
    cal = dict(np.load(os.path.join(d, "camera_calibration.npz")))
    cal["refractory_period"] = np.array(250000)            # ns, i64 like the calibration files
    np.savez(os.path.join(d, "camera_calibration.npz"), **cal)
    torch.save(torch.tensor(1000000), os.path.join(d, "max_refractory_period.pt"))
    ct = egp.ContrastThreshold(d, parameterize_mean_ct=True)
    rp = egp.RefractoryPeriod(d)
    with torch.no_grad():  # move off the calibrated values so the parametrisations matter
        ct.parametrizations.p2n_contrast_threshold_ratio.original.add_(0.07)
        ct.parametrizations.mean_contrast_threshold.original.sub_(0.03)
        rp.parametrizations._refractory_period.original.add_(12345.678)
    code = compile(_training_step_ts_code(), "deblur_e_nerf.py:418-455", "exec")
    g = torch.Generator().manual_seed(21)
    N = 512
    num_pos = torch.randint(0, 3, (N,), generator=g)
    num_neg = torch.randint(0, 3, (N,), generator=g)
    num_pos[:128] = (torch.rand(128, generator=g) < 0.5).long()      # queued events: one per interval
    num_neg[:128] = 1 - num_pos[:128]
    end_ts = (torch.rand(N, generator=g, dtype=torch.float64) * 9e8 + 1e8).floor().long()
    start_ts = end_ts - (torch.rand(N, generator=g, dtype=torch.float64) * 3e6 + 3e5).floor().long()
    norm = torch.rand(4, N, generator=g, dtype=torch.float64)
    norm[0, :256] = 1.0                                                # Dirac(1) interval sampler
    norm[1, :8] = torch.tensor([0.0, 0.5, 1.0, 0.25, 0.75, 1e-9, 1 - 1e-9, 0.5 - 1e-12], dtype=torch.float64)
    norm[3, :8] = norm[1, :8]
    out = dict(num_pos=num_pos.numpy(), num_neg=num_neg.numpy(), end_ts=end_ts.numpy(), start_ts=start_ts.numpy(),
               norm=norm.numpy(), pos_ct=ct.pos_contrast_threshold.detach().numpy(),
               neg_ct=ct.neg_contrast_threshold.detach().numpy(),
               mean_ct=ct.mean_contrast_threshold.detach().numpy(),
               refractory_period=rp.refractory_period.detach().numpy())
    for tag, wd, wt in (("both", 1.0, 1e-3), ("diff", 1.0, 0.0), ("tv", 0.0, 1e-3)):
        ev = ED(num_pos=num_pos.clone(), num_neg=num_neg.clone(), end_ts=end_ts.clone(), start_ts=start_ts.clone())
        batch = ED(event=ev, normalized=ED(ts_diff=norm[0], diff_start_ts=norm[1], ts_subdiff=norm[2],
                                           subdiff_start_ts=norm[3]))
        with torch.no_grad():
            batch.event = ct(batch.event)
            batch.event = rp(batch.event)
            self_ = types.SimpleNamespace(hparams=ED(loss=ED(weight=ED(log_intensity_diff=wd, log_intensity_tv=wt))))
            exec(code, {"torch": torch}, {"batch": batch, "self": self_})
        out[f"{tag}:lid"] = batch.event.log_intensity_diff.numpy()
        out[f"{tag}:start_ts"] = batch.event.start_ts.numpy()
        for grp in ("diff", "subdiff"):
            if batch[grp] is not None:
                for k in ("ts_diff", "start_ts", "end_ts"):
                    out[f"{tag}:{grp}.{k}"] = batch[grp][k].numpy()
    save("events.npz", **out)


def gen_rays():
    nerfm = _refload.load("models.nerf")
    g = torch.Generator().manual_seed(23)
    N, M = 400, 4
    K = torch.tensor([[1111.0, 0.0, 400.0], [0.0, 1111.0, 400.0], [0.0, 0.0, 1.0]])
    K_inv = torch.linalg.inv(K)
    pixel = torch.rand(N, 2, generator=g) * 800
    pixel[:4] = torch.tensor([[0.0, 0.0], [799.5, 799.5], [400.0, 400.0], [0.5, 799.0]])
    q, _ = torch.linalg.qr(torch.randn(M, N, 3, 3, generator=g, dtype=torch.float64))
    rot = (q * torch.sign(torch.linalg.det(q))[..., None, None]).float()      # proper rotations
    pos = torch.randn(M, N, 3, generator=g) * 4
    o, dr = nerfm.NeRF.pixel_params_to_ray(K_inv, pixel, pos, rot)          # (N,2) pixels broadcast over M
    o1, d1 = nerfm.NeRF.pixel_params_to_ray(K_inv, pixel, pos[0], rot[0])
    save("rays.npz", K_inv=K_inv.numpy(), pixel=pixel.numpy(), T_wc_position=pos.numpy(),
         T_wc_orientation=rot.numpy(), ray_origin=o.numpy(), ray_direction=dr.numpy(),
         ray_origin_1=o1.numpy(), ray_direction_1=d1.numpy())


# ----------------------------------------------------------------------------
RENDER_CFG = dict(aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], near=1.43, far=6.63, res=24,
                  step=float(np.sqrt(3) * 3.0 / 1024))  # synthetic.yaml nerf section, render_step_size "auto"
ARCH = dict(net_depth=8, net_width=256, skip_layer=4, net_depth_condition=1, net_width_condition=128,
            hidden_activation="softplus", density_activation="shifted_trunc_exp", radiance_activation="softplus",
            pos_encoder_max_deg=10, view_encoder_max_deg=4, weight_norm=False)


def _chair_rays(R, seed):
    g = torch.Generator().manual_seed(seed)
    v = torch.randn(R, 3, generator=g)
    o = v / v.norm(dim=-1, keepdim=True) * 4.03
    d = -o / o.norm(dim=-1, keepdim=True) + (torch.rand(R, 3, generator=g) * 2 - 1) * np.sin(0.3)
    d = d / d.norm(dim=-1, keepdim=True)
    return o.float(), d.float()


def _grad_pick(nerf, n_pick=4096, seed=77):
    """Gradient summary small enough for a fixture: every bias, three whole weight tensors and a
    seeded subset of the flat MLP gradient (reference named_parameters() order)."""
    out = {}
    flat = []
    for k, p in nerf.radiance_field.mlp.named_parameters():
        gr = p.grad.detach().reshape(-1)
        flat.append(gr)
        if k.endswith("bias") or k in ("base.hidden_layers.0.weight", "sigma_layer.output_layer.weight",
                                       "rgb_layer.output_layer.weight"):
            out[f"grad:{k}"] = gr.numpy()
    flat = torch.cat(flat)
    idx = torch.randperm(flat.numel(), generator=torch.Generator().manual_seed(seed))[:n_pick].sort().values
    out["grad_pick_idx"] = idx.numpy()
    out["grad_pick"] = flat[idx].numpy()
    out["grad_norm"] = np.array(float(flat.double().norm()))
    return out


def _ref_nerf(rd, seed, res):
    """The reference NeRF (models/nerf.py) in the chair configuration with the nerfacc stand-in
    (oracle/nerfacc.py); weights = PyTorch default Linear init under torch.manual_seed(seed)."""
    nerfm = _refload.load("models.nerf")
    ED = sys.modules["easydict"].EasyDict
    CT = sys.modules["nerfacc"].ContractionType
    c = RENDER_CFG
    torch.manual_seed(seed)
    occ = ED(resolution=res, occ_thre=0.01, ema_decay=0.95, warmup_steps=256, n=16)
    return nerfm.NeRF(c["aabb"], CT.AABB, occ, c["near"], c["far"], c["step"], "parameter", 0.0, 1e-4, 0.0, 16384,
                      "mlp", ED(ARCH), 3, rd)


def gen_render(rd=1, seed=4, R=64, sigma_bias_shift=3.5):
    """render.npz -- the reference's NeRF.forward (models/nerf.py:230-286) -> external/utils.py
    render_image (the sigma_fn / rgb_sigma_fn closures, chunking) -> vol_rendering.rendering
    (weights, three accumulations, background) in the chair configuration (synthetic.yaml), with
    nerfacc's marching / scan / grid restated by oracle/nerfacc.py: the occupancy-grid update at
    step 0, a training-mode forward (stratified; the jitter is recorded), its backward, and an
    eval-mode forward."""
    nerf = _ref_nerf(rd, seed, RENDER_CFG["res"])
    from oracle import nerfacc as onerfacc
    out = dict(seed=seed, rd=rd, res=RENDER_CFG["res"], step=RENDER_CFG["step"], aabb=np.array(RENDER_CFG["aabb"]),
               near=RENDER_CFG["near"], far=RENDER_CFG["far"], sigma_bias_shift=sigma_bias_shift)
    o, d = _chair_rays(R, 31)
    out.update(rays_o=o.numpy(), rays_d=d.numpy())
    nerf.train()
    torch.manual_seed(100)
    nerf.update_occ_grid(step=0, T_wc_position=o)
    grid = nerf.occupancy_grid
    out.update(occ_u=grid.last_u.numpy(), occs=grid.occs.numpy(), binary=grid.binary.numpy())
    # the renders below use a denser field (rays saturate, so the early stop T < 1e-4 drops samples)
    # and a structured grid (a ball of occupied cells with holes), so the DDA skip is exercised
    with torch.no_grad():
        nerf.radiance_field.mlp.sigma_layer.output_layer.bias.add_(sigma_bias_shift)
    r = RENDER_CFG["res"]
    c = (torch.stack(torch.meshgrid(*[torch.arange(r)] * 3, indexing="ij"), -1).float() + 0.5) / r - 0.5
    ball = (c.norm(dim=-1) < 0.4) & ~((c[..., 0] > 0.1) & (c[..., 1].abs() < 0.1))
    grid._binary = ball
    out["binary_render"] = ball.numpy()
    g = torch.Generator().manual_seed(41)
    g_rad, g_op, g_dp = torch.randn(R, generator=g), torch.randn(R, generator=g), torch.randn(R, generator=g)
    if rd > 1:
        g_rad = torch.randn(R, rd, generator=g)
    torch.manual_seed(101)
    rad, op, dp, mspr = nerf(o, d)
    LAST = onerfacc.LAST
    out.update(train_jitter=LAST["jitter"].numpy(), train_marched_ri=LAST["marched"][0],
               train_marched_t0=LAST["marched"][1], train_marched_t1=LAST["marched"][2],
               train_t_min=LAST["t_min"], train_t_max=LAST["t_max"],
               train_kept_ri=LAST["kept"][0].numpy(), train_kept_t0=LAST["kept"][1][:, 0].numpy(),
               train_kept_t1=LAST["kept"][2][:, 0].numpy(), train_prepass_sigma=LAST["prepass_sigma"],
               train_radiance=rad.detach().numpy(), train_opacity=op.detach().numpy(),
               train_depth=dp.detach().numpy(), train_mspr=np.array(mspr),
               g_rad=g_rad.numpy(), g_op=g_op.numpy(), g_dp=g_dp.numpy())
    ((rad * g_rad).sum() + (op * g_op).sum() + (dp * g_dp).sum()).backward()
    out.update(_grad_pick(nerf))
    out["grad_bkgd_orig"] = nerf.parametrizations.render_bkgd.original.grad.numpy()
    nerf.eval()
    with torch.no_grad():
        rad, op, dp, mspr = nerf(o, d)
    out.update(eval_radiance=rad.numpy(), eval_opacity=op.numpy(), eval_depth=dp.numpy(), eval_mspr=np.array(mspr),
               eval_kept_ri=LAST["kept"][0].numpy(), eval_kept_t0=LAST["kept"][1][:, 0].numpy())
    # the reference's own rendering() on explicit packed samples (vol_rendering.py:16-128)
    vr = _refload.load("external.vol_rendering")
    n = 300
    ri = torch.sort(torch.randint(0, 20, (n,), generator=g)).values.int()
    ts = torch.rand(n, 1, generator=g) * 3 + 1.5
    te = ts + torch.rand(n, 1, generator=g) * 0.05 + 1e-3
    sig = (torch.rand(n, 1, generator=g) * 30).requires_grad_(True)
    rgb = torch.rand(n, rd, generator=g).requires_grad_(True)
    bk = torch.tensor([0.7] * rd, requires_grad=True)
    col, opa, dep = vr.rendering(ts, te, ri, 24, rgb_sigma_fn=lambda a, b, c: (rgb, sig), render_bkgd=bk)
    gc, go, gd = torch.randn(24, rd, generator=g), torch.randn(24, 1, generator=g), torch.randn(24, 1, generator=g)
    ((col * gc).sum() + (opa * go).sum() + (dep * gd).sum()).backward()
    out.update(vr_ri=ri.numpy(), vr_t0=ts.numpy(), vr_t1=te.numpy(), vr_sigma=sig.detach().numpy(),
               vr_rgb=rgb.detach().numpy(), vr_bkgd=bk.detach().numpy(), vr_color=col.detach().numpy(),
               vr_opacity=opa.detach().numpy(), vr_depth=dep.detach().numpy(), vr_gc=gc.numpy(), vr_go=go.numpy(),
               vr_gd=gd.numpy(), vr_dsigma=sig.grad.numpy(), vr_drgb=rgb.grad.numpy(), vr_dbkgd=bk.grad.numpy())
    save(f"render_rd{rd}.npz", **out)


def gen_fixed(rd=1, seed=4, R=64, S=128, sigma_bias_shift=0.0):
    """fixed_rd*.npz -- the benchmark's fixed-count sampler (S stratified samples
    t = t_min + (k + u) dt in AABB n [near, far], oracle/nerf.stratified_samples) packed as nerfacc
    samples and rendered by the reference's own glue: the rgb_sigma_fn closure of external/utils.py
    (positions o + d (t0 + t1) / 2, view directions d) over its VanillaNeRFRadianceField, then
    external/vol_rendering.rendering (weights, accumulation, background); colour / opacity / depth
    and the gradients of a random projection of them."""
    from oracle import nerf as onerf
    nerf = _ref_nerf(rd, seed, RENDER_CFG["res"])
    rf = nerf.radiance_field
    with torch.no_grad():
        rf.mlp.sigma_layer.output_layer.bias.add_(sigma_bias_shift)
    o, d = _chair_rays(R, 33)
    u = torch.rand(R, generator=torch.Generator().manual_seed(34))
    t0, t1 = onerf.stratified_samples(o, d, u, torch.tensor(RENDER_CFG["aabb"]), RENDER_CFG["near"],
                                      RENDER_CFG["far"], S)
    ri = torch.arange(R, dtype=torch.int32).repeat_interleave(S)
    ts, te = t0.reshape(-1, 1), t1.reshape(-1, 1)
    vr = _refload.load("external.vol_rendering")

    def rgb_sigma_fn(t_starts, t_ends, ray_indices):
        ray_indices = ray_indices.long()
        pos = o[ray_indices] + d[ray_indices] * (t_starts + t_ends) / 2.0
        return rf(pos, d[ray_indices])
    bk = torch.tensor([0.7] * rd, requires_grad=True)
    col, opa, dep = vr.rendering(ts, te, ri, R, rgb_sigma_fn=rgb_sigma_fn, render_bkgd=bk)
    g = torch.Generator().manual_seed(35)
    gc, go, gd = torch.randn(R, rd, generator=g), torch.randn(R, 1, generator=g), torch.randn(R, 1, generator=g)
    ((col * gc).sum() + (opa * go).sum() + (dep * gd).sum()).backward()
    out = dict(seed=seed, rd=rd, S=S, sigma_bias_shift=sigma_bias_shift, aabb=np.array(RENDER_CFG["aabb"]),
               near=RENDER_CFG["near"], far=RENDER_CFG["far"], rays_o=o.numpy(), rays_d=d.numpy(), jitter=u.numpy(),
               color=col.detach().numpy(), opacity=opa.detach().numpy(), depth=dep.detach().numpy(), gc=gc.numpy(),
               go=go.numpy(), gd=gd.numpy(), grad_bkgd=bk.grad.numpy())
    out.update(_grad_pick(nerf))
    save(f"fixed_rd{rd}.npz", **out)


def gen_fixed_all():
    gen_fixed(1, seed=4)
    gen_fixed(3, seed=5)


def gen_traj():
    """traj.npz -- models/trajectories.py LinearTrajectory (searchsorted, lerp, the shortest-path
    full-angle slerp of utils/tensor_ops.py:118-184, quaternion -> rotation matrix) with RoMa
    1.2.7 restated by oracle/roma.py."""
    trm = _refload.load("models.trajectories")
    ED = sys.modules["easydict"].EasyDict
    g = torch.Generator().manual_seed(51)
    C = 40
    ts = torch.cumsum(torch.randint(1_000_000, 5_000_000, (C,), generator=g), 0) + 100_000_000   # i64 ns
    pos = torch.cumsum(torch.randn(C, 3, generator=g) * 0.05, 0) + torch.tensor([0.0, 0.0, 4.0])
    q = torch.randn(C, 4, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    # small steps between consecutive orientations, a few sign flips (shortest path) and a near-pi pair
    for i in range(1, C):
        q[i] = q[i - 1] + torch.randn(4, generator=g) * 0.05
        q[i] = q[i] / q[i].norm()
    q[7] = -q[7]
    q[20] = -q[20]
    q[30] = q[29] + torch.tensor([0.0, 0.0, 0.0, 1e-5])
    q[30] = q[30] / q[30].norm()
    cp = ED(camera_poses=ED(T_wc_position=pos, T_wc_orientation=q, T_wc_timestamp=ts))
    traj = trm.LinearTrajectory(cp)
    N = 600
    qt = ts[0].double() + torch.rand(N, generator=g, dtype=torch.float64) * float(ts[-1] - ts[0])
    qt[:4] = torch.tensor([float(ts[0]), float(ts[-1]), float(ts[5]), float(ts[5]) + 0.5], dtype=torch.float64)
    p_out, r_out = traj(qt)
    qt2 = qt[:480].reshape(16, 30)
    p2, r2 = traj(qt2)
    save("traj.npz", T_wc_position=pos.numpy(), T_wc_orientation=q.numpy(), T_wc_timestamp=ts.numpy(),
         query_ts=qt.numpy(), position=p_out.numpy(), rotation=r_out.numpy(), query_ts_2d=qt2.numpy(),
         position_2d=p2.numpy(), rotation_2d=r2.numpy())


# ----------------------------------------------------------------------------
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


def write_dataset(d, cal, poses, max_refractory_period=1_000_000):
    np.savez(os.path.join(d, "camera_calibration.npz"), **cal)
    np.savez(os.path.join(d, "camera_poses.npz"), **poses)
    torch.save(torch.tensor(max_refractory_period), os.path.join(d, "max_refractory_period.pt"))


def synthetic_event_batch(N, S, seed, img=800, ts_lo=1.5e8, ts_hi=9.5e8):
    """A reference-shaped training batch (datamodule.py:215-247): events (1, N, ...) and the
    normalized samples (1, N) / (1, S - 1, N)."""
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
    if S:
        nz["interval_gen"] = torch.full((1, S - 1, N), 0.5, dtype=torch.float64)
    return dict(event=ev, normalized=nz)


STEP_DEFAULT = dict(rd=1, pixbw=False, S=8, arch="mlp", N=40, contraction="aabb", aabb=None, near=None, far=None,
                    cone=0.0, res=24, tv=1e-3, pixbw_free=False)


def _step_cfg(**kw):
    c = dict(STEP_DEFAULT, **kw)
    rc = RENDER_CFG
    c["aabb"] = list(rc["aabb"]) if c["aabb"] is None else list(c["aabb"])
    c["near"] = rc["near"] if c["near"] is None else c["near"]
    c["far"] = rc["far"] if c["far"] is None else c["far"]
    # render_step_size "auto" (deblur_e_nerf.py:277-283): sqrt(3) max extent / 1024
    a = np.asarray(c["aabb"], np.float64)
    c["step"] = float(np.sqrt(3) * float((a[3:] - a[:3]).max()) / 1024)
    return c


def ref_deblur_step_module(d, seed, cfg, ct_free=True, refr_free=True):
    """The reference DeblurENeRF's training-path methods bound to a module assembled from the
    reference's own components (the constructor needs eval images and Lightning)."""
    dm = _refload.load("models.deblur_e_nerf")
    egp = _refload.load("models.event_generation_params")
    pbm = _refload.load("models.pixel_bandwidth")
    trm = _refload.load("models.trajectories")
    lossm = _refload.load("loss_metric.loss")
    ED = sys.modules["easydict"].EasyDict
    datasets = _refload.load("data.datasets")
    rd, pixbw, S = cfg["rd"], cfg["pixbw"], cfg["S"]
    m = dm.DeblurENeRF.__new__(dm.DeblurENeRF)
    torch.nn.Module.__init__(m)
    m.hparams = ED(min_modeled_intensity=0.001,
                   contrast_threshold=ED(parameterize_mean_ct=True, freeze=not ct_free),
                   refractory_period=ED(freeze=not refr_free),
                   pixel_bandwidth=ED(enable=pixbw, it_sample_size=S, f_c_dominant_min=21,
                                      target_cumprob=ED(max_sample_lifetime=0.95)),
                   loss=ED(weight=ED(log_intensity_diff=1.0, log_intensity_tv=cfg["tv"], nerf_mlp_weight_decay=1e-6),
                           error_fn=ED(log_intensity_diff="huber", log_intensity_tv="l1"),
                           normalize=ED(log_intensity_diff=True, log_intensity_tv=True)))
    cal = datasets.Event.load_camera_calibration(d)
    m.has_bayer_filter = str(cal["bayer_pattern"]) != ""
    m.register_buffer("train_intrinsics_inv", torch.linalg.inv(torch.from_numpy(cal["intrinsics"])), persistent=False)
    m.render_bkgd = "parameter"
    m.train_ray_sample_batch_size = 131072
    m.MODEL_COMPONENTS = ["contrast_threshold", "refractory_period", "nerf"]
    m.MULTI_PARAM_MODEL_COMPONENTS = ["contrast_threshold"]
    m.contrast_threshold = egp.ContrastThreshold(d, True)
    m.refractory_period = egp.RefractoryPeriod(d)
    cp = datasets.CameraPose(d, None)
    if pixbw:
        m.pixel_bandwidth = pbm.PixelBandwidth(d, cp.camera_poses.T_wc_timestamp.min(), 21,
                                               ED(max_sample_lifetime=0.95))
        m.MODEL_COMPONENTS.append("pixel_bandwidth")
        m.MULTI_PARAM_MODEL_COMPONENTS.append("pixel_bandwidth")
        for p in m.pixel_bandwidth.parameters():
            p.requires_grad_(bool(cfg["pixbw_free"]))
    m.nerf = _ref_nerf(rd, seed, cfg["res"]) if cfg["arch"] == "mlp" else _ref_nerf_ngp(rd, seed, cfg["res"], cfg)[0]
    m.trajectory = trm.LinearTrajectory(cp)
    for c, free in (("contrast_threshold", ct_free), ("refractory_period", refr_free)):
        for p in getattr(m, c).parameters():
            p.requires_grad_(free)
    m.loss = lossm.Loss(m.hparams.loss.weight, m.hparams.loss.error_fn, m.hparams.loss.normalize)
    sampler = types.SimpleNamespace(size=1)
    m.trainer = types.SimpleNamespace(accumulate_grad_batches=1, datamodule=types.SimpleNamespace(
        train_dataset=types.SimpleNamespace(batch_size=1),
        train_normalized_sampler=types.SimpleNamespace(datasets=[sampler])))
    m.global_step = 0
    m.log = lambda *a, **k: None
    m.all_gather = lambda t: t[None]
    return m


def _step_grads(m, cfg):
    """The gradients a step fixture records (the reference's parameter names)."""
    out = {}
    if cfg["arch"] == "mlp":
        out.update(_grad_pick(m.nerf))
    else:
        out.update({f"grad:{k}": prm.grad.detach().numpy() for k, prm in m.nerf.radiance_field.named_parameters()})
    out["grad_bkgd_orig"] = m.nerf.parametrizations.render_bkgd.original.grad.numpy()
    ctp = m.contrast_threshold.parametrizations
    out["d_p2n_orig"] = ctp.p2n_contrast_threshold_ratio.original.grad.numpy()
    out["d_mean_ct_orig"] = ctp.mean_contrast_threshold.original.grad.numpy()
    out["dtau_orig"] = m.refractory_period.parametrizations._refractory_period.original.grad.numpy()
    if cfg["pixbw"] and cfg["pixbw_free"]:
        for name in ("tau_mil_it_eff_prod", "A_amp_inv", "A_loop_inv", "tau_out", "tau_sf", "tau_diff"):
            out[f"dpixbw:{name}"] = getattr(m.pixel_bandwidth.parametrizations, name).original.grad.numpy()
    return out


class _GradTap(torch.autograd.Function):
    """Identity whose backward hands the incoming gradient to ``fn``."""

    @staticmethod
    def forward(ctx, x, fn):
        ctx.fn = fn
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.fn(g)
        return g, None


N_PERM = 3  # event-permuted f32 reruns of each step fixture


def gen_step(pixbw=False, rd=1, seed=6, N=40, S=8, tag=None, arch="mlp", **extra):
    """step_*.npz -- the reference DeblurENeRF.training_step (deblur_e_nerf.py:396-586) run on a
    reference-shaped batch: event correction, supervision timestamps, the occupancy-grid update,
    render_log_intensity x 4 (trajectory, rays, NeRF.forward through render_image with the nerfacc
    stand-in; the pixel-bandwidth model when on), update_train_batch_size, Loss.compute; then the
    backward.  Contrast thresholds and refractory period learnable (07_ziggy_and_fuzz_hdr.yaml:172).
    Three runs of the same step:
      * "full": the reference as configured (f32) -- the fixture's main values;
      * "nopose": the trajectory's interpolation weight detached (``dtau_orig_nopose``: the part of the
        tau_r gradient that does not flow through the camera pose);
      * "f64": the whole module and batch in float64 on the f32 run's recorded occupancy grid and
        marched samples (``*_f64``): the reference's own f32 rounding error, the floor of the
        tolerances in tests/test_deblur_gpu.py."""
    from oracle import nerfacc as onerfacc
    cfg = _step_cfg(pixbw=pixbw, rd=rd, S=S, arch=arch, N=N, **extra)
    cal, poses = synthetic_dataset_arrays(rd)
    d = tempfile.mkdtemp(prefix="den_step_")
    write_dataset(d, cal, poses)
    batch = synthetic_event_batch(N, S if pixbw else 0, seed + 100)
    out = dict(rd=rd, seed=seed, N=N, S=S, pixbw=pixbw, res=cfg["res"], sigma_bias_shift=2.0, arch=np.array(arch),
               contraction=np.array(cfg["contraction"]), aabb=np.array(cfg["aabb"], np.float32), near=cfg["near"],
               far=cfg["far"], cone=cfg["cone"], tv=cfg["tv"], pixbw_free=cfg["pixbw_free"],
               **{f"cal:{k}": v for k, v in cal.items()}, **{f"pose:{k}": v for k, v in poses.items()},
               **{f"event:{k}": v.numpy() for k, v in batch["event"].items()},
               **{f"normalized:{k}": v.numpy() for k, v in batch["normalized"].items()})
    kept = []
    real = onerfacc.ray_marching
    for variant in ("full", "nopose", "f64") + tuple(f"f32p{k}" for k in range(N_PERM)):
        m = ref_deblur_step_module(d, seed, cfg)
        dmod = sys.modules["deblur_e_nerf.external.utils"]
        with torch.no_grad():
            if arch == "mlp":
                m.nerf.radiance_field.mlp.sigma_layer.output_layer.bias.add_(2.0)
            else:
                m.nerf.radiance_field.mlp_base[1].output_layer.bias[0] += 2.0
        m.train()
        b = {k: {kk: vv.clone() for kk, vv in v.items()} for k, v in batch.items()}
        jit = []
        perm = inv = None
        if variant.startswith("f32p"):
            # the same step with the events in another order: every sum over events / rays / samples
            # runs in another order, the f64 result does not change -- the spread of these f32 runs is
            # the reference's own f32 rounding noise (tests/test_deblur_gpu.py bounds)
            perm = torch.randperm(N, generator=torch.Generator().manual_seed(400 + int(variant[4:])))
            inv = torch.argsort(perm)
            b = {k: {kk: vv[..., perm].clone() if kk != "position" else vv[:, perm].clone() for kk, vv in v.items()}
                 for k, v in b.items()}
        if variant == "f64":
            m.double()
            b["event"]["position"] = b["event"]["position"].double()
        if variant != "full" and variant != "nopose":
            grid = m.nerf.occupancy_grid

            def replay_grid(step, T_wc_position, g=grid):
                g.occs.copy_(torch.from_numpy(out["occs"]))
                g._binary.copy_(torch.from_numpy(out["binary"]))
            m.nerf.update_occ_grid = replay_grid
            calls = iter(kept)

            def rec(*a, _inv=inv, **k):
                ri, t0, t1 = (t.clone() for t in next(calls))
                if _inv is not None:  # ray s N + e of the original order is ray s N + inv[e] here
                    r = ri.long()
                    new = (r // N) * N + _inv[r % N]
                    order = torch.sort(new, stable=True).indices
                    ri, t0, t1 = new[order].to(ri.dtype), t0[order], t1[order]
                return ri, t0, t1
        else:
            def rec(*a, **k):
                r = real(*a, **k)
                jit.append(onerfacc.LAST["jitter"].clone())
                if variant == "full":
                    kept.append(tuple(t.clone() for t in r))
                return r
        if variant == "nopose":
            orig_forward = type(m.trajectory).forward
            m.trajectory.forward = lambda ts, f=orig_forward, t=m.trajectory: f(t, ts.detach())
        dmod.ray_marching = rec
        # d loss / d render timestamps of each render_log_intensity call, the part that flows
        # through the call itself (trajectory -> rays -> render, the pose path's input): an identity
        # in front of the call records it, the timestamp's other uses (diff end / subdiff
        # timestamps derived from it) do not reach it
        dts = []
        orig_rli = m.render_log_intensity

        def rli(timestamp, *a, _f=orig_rli, **k):
            if timestamp.requires_grad:
                slot = len(dts)
                dts.append(None)
                timestamp = _GradTap.apply(timestamp, lambda g, i=slot: dts.__setitem__(i, g.detach().clone()))
            return _f(timestamp, *a, **k)
        m.render_log_intensity = rli
        # per render_log_intensity call: its log intensities (the TV term's |end - start| decides
        # which events have a well-defined L1 sign); per NeRF.forward call: d loss / d colour x
        # (1 - opacity) per ray, the terms the render background's gradient sums
        lis, bkray = [], []

        def rli_rec(*a, _f=m.render_log_intensity, **k):
            r = _f(*a, **k)
            lis.append(r[0].detach().clone())
            return r
        m.render_log_intensity = rli_rec
        orig_nerf_forward = m.nerf.forward

        def nerf_rec(o, dr, _f=orig_nerf_forward):
            rad, op, dp, mspr = _f(o, dr)
            slot = len(bkray)
            bkray.append(None)
            keep = (1 - op.detach()).clone()
            rad = _GradTap.apply(rad, lambda g, i=slot, w=keep: bkray.__setitem__(
                i, (g.detach() * (w[..., None] if g.dim() > w.dim() else w)).clone()))
            return rad, op, dp, mspr
        m.nerf.forward = nerf_rec
        # the occupancy update's torch.randint draws (the cone branch's random camera per point,
        # nerf.py:178-181), replayed by tests through models/nerf._randint
        cam_draws = []
        real_randint = torch.randint

        def randint_rec(*a, **k):
            r = real_randint(*a, **k)
            cam_draws.append(r.clone())
            return r
        orig_upd = m.nerf.update_occ_grid

        def upd_rec(*a, _f=orig_upd, **k):
            torch.randint = randint_rec
            try:
                return _f(*a, **k)
            finally:
                torch.randint = real_randint
        m.nerf.update_occ_grid = upd_rec
        torch.manual_seed(200)
        try:
            loss = m.training_step(b, 0)
            loss.backward()
        finally:
            dmod.ray_marching = real
            torch.randint = real_randint
        if variant in ("full", "f64"):
            sfx = "" if variant == "full" else "_f64"
            out.update({f"li_g{i}{sfx}": li.numpy() for i, li in enumerate(lis)})
            out.update({f"bkray_{i}{sfx}": g.numpy() for i, g in enumerate(bkray) if g is not None})
        if variant != "nopose":
            sfx = "" if variant == "full" else "_" + variant
            # per-event timestamp gradients back in the original event order
            out.update({f"dts_g{i}{sfx}": (g if inv is None else g[..., inv]).numpy() for i, g in enumerate(dts)
                        if g is not None})
        if variant == "full":
            grid = m.nerf.occupancy_grid
            if cam_draws:
                out.update({f"occ_randint_{i}": r.numpy() for i, r in enumerate(cam_draws)})
            out.update(occ_u=grid.last_u.numpy(), occs=grid.occs.numpy(), binary=grid.binary.numpy(),
                       loss=loss.detach().numpy(), mspr=np.array(float(m.train_batch_size) if hasattr(
                           m, "train_batch_size") else 0.0),
                       new_batch_size=np.array(m.trainer.datamodule.train_dataset.batch_size),
                       **{f"jitter_{i}": j.numpy() for i, j in enumerate(jit)})
            out.update(_step_grads(m, cfg))
            if arch != "mlp":
                rf = m.nerf.radiance_field
                out.update({f"param:{k}": prm.detach().numpy() for k, prm in rf.named_parameters()
                            if k != "mlp_base.0.params"})
                out["table"] = rf.mlp_base[0].params.detach().numpy()
                out["pos_encoding"] = np.array(json.dumps(NGP_SMALL))
        elif variant == "nopose":
            out["dtau_orig_nopose"] = m.refractory_period.parametrizations._refractory_period.original.grad.numpy()
            out["loss_nopose"] = loss.detach().numpy()
        else:
            sfx = "_" + variant
            out["loss" + sfx] = loss.detach().numpy()
            for k, v in _step_grads(m, cfg).items():
                if k != "grad_pick_idx":
                    out[k + sfx] = v
    save(tag or f"step_{'pixbw' if pixbw else 'nopixbw'}_rd{rd}.npz", **out)


def gen_eval(rd=1, seed=6, H=20, W=24):
    """eval_rd*.npz -- the reference DeblurENeRF.evaluation_step's render (deblur_e_nerf.py:602-652):
    render_pixels of an H x W image (the meshgrid pixel positions of :120-127) at one camera pose,
    eval mode (no jitter, chunked marching), after one occupancy-grid update at step 0 (its U[0,1)
    draws recorded).  Small intrinsics (f = 1.4 W) so the image covers the AABB."""
    cfg = _step_cfg(rd=rd)
    cal, poses = synthetic_dataset_arrays(rd)
    d = tempfile.mkdtemp(prefix="den_eval_")
    write_dataset(d, cal, poses)
    m = ref_deblur_step_module(d, seed, cfg)
    with torch.no_grad():
        m.nerf.radiance_field.mlp.sigma_layer.output_layer.bias.add_(2.0)
    torch.manual_seed(300)
    m.nerf.update_occ_grid(step=0, T_wc_position=m.trajectory.T_wc_position)
    grid = m.nerf.occupancy_grid
    m.eval()
    K = torch.tensor([[1.4 * W, 0.0, W / 2.0], [0.0, 1.4 * W, H / 2.0], [0.0, 0.0, 1.0]])
    kinv = torch.linalg.inv(K)
    i = 17
    pos = m.trajectory.T_wc_position[i]
    from oracle import roma as oroma
    rot = oroma.unitquat_to_rotmat(m.trajectory.T_wc_orientation_quat[i])
    pix = torch.stack(torch.meshgrid(torch.arange(W), torch.arange(H), indexing="xy"), dim=2).to(torch.float32)
    P = pos.view(1, 1, 3).expand(H, W, -1)
    R = rot.view(1, 1, 3, 3).expand(H, W, -1, -1)
    with torch.no_grad():
        img, opacity, depth, mspr, _ = m.render_pixels(kinv, pix, P, R)
    save(f"eval_rd{rd}.npz", rd=rd, seed=seed, N=0, S=8, pixbw=False, res=cfg["res"], sigma_bias_shift=2.0,
         **{f"cal:{k}": v for k, v in cal.items()}, **{f"pose:{k}": v for k, v in poses.items()},
         occ_u=grid.last_u.numpy(), occs=grid.occs.numpy(), kinv=kinv.numpy(), pos=pos.detach().numpy(),
         rot=rot.detach().numpy(), H=H, W=W, img=img.numpy(), opacity=opacity.numpy(), depth=depth.numpy(),
         mean_samples_per_ray=np.array(float(mspr)))


def gen_eval_all():
    gen_eval(1, seed=6)
    gen_eval(3, seed=8)


def gen_step_pixbw():
    gen_step(True, 1)


def gen_step_nopixbw():
    gen_step(False, 1)


def gen_mlp_density():
    """The other density activations of models/nerf.py:20-29 (mip-NeRF's shifted_softplus,
    softplus), through the reference's VanillaNeRFRadianceField."""
    gen_mlp(1, seed=4, density="shifted_softplus")
    gen_mlp(3, seed=5, density="softplus")


def gen_mlp_unbounded():
    gen_mlp(3, seed=2, contraction="sphere")
    gen_mlp(1, seed=3, contraction="tanh")


# ----------------------------------------------------------------------------
NGP_SMALL = dict(otype="HashGrid", n_levels=8, n_features_per_level=2, log2_hashmap_size=12, base_resolution=16,
                 per_level_scale=1.4472692012786865, interpolation="Linear")
NGP_ARCH = dict(pos_encoding=dict(NGP_SMALL), dir_encoding=dict(degree=4),
                mlp_base=dict(hidden_activation="softplus", density_activation="shifted_trunc_exp", n_neurons=64,
                              n_hidden_layers=1, geo_feat_dim=15, weight_norm=False),
                mlp_head=dict(hidden_activation="softplus", radiance_activation="softplus", n_neurons=64,
                              n_hidden_layers=2, weight_norm=False))


def gen_ngp(rd=1, seed=21, cfg="small", contraction="aabb", hidden="softplus", radiance="softplus", n=512,
            density="shifted_trunc_exp"):
    """ngp_*.npz -- the reference's NGPradianceField (external/ngp.py:109-280: contraction, the
    mlp_base / mlp_head MLPs of external/mlp.py, SHEncoder, shifted_trunc_exp, the configured
    activations of models/nerf.py:17-29) forward + backward, with oracle/tcnn.py standing in for
    tcnn.Encoding (tiny-cuda-nn is absent: the grid encoding itself is parity unpinned).
    cfg "small": 8 levels of 2^12 entries (dense level 0, hashed levels 1..7; the table and its
    whole gradient are stored); cfg "default": configs/train/synthetic.yaml's 16 levels of 2^19
    (the table is regenerated from the seed by oracle/ngp.build_params, the fixture keeps its
    f64 sum and the gradient's nonzero entries)."""
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from oracle import ngp as ongp
    from oracle import tcnn as otcnn
    ngp = _refload.load("external.ngp")
    sys.modules["tinycudann"].Encoding = otcnn.Encoding
    ContractionType = sys.modules["nerfacc"].ContractionType
    ctype = {"aabb": ContractionType.AABB, "sphere": ContractionType.UN_BOUNDED_SPHERE,
             "tanh": ContractionType.UN_BOUNDED_TANH}[contraction]
    pos = dict(NGP_SMALL) if cfg == "small" else dict(ongp.POS_ENCODING)
    act = {"softplus": torch.nn.Softplus(beta=100), "relu": torch.nn.ReLU()}
    ract = {"softplus": torch.nn.Softplus(beta=1), "sigmoid": torch.nn.Sigmoid()}
    nerfm = _refload.load("models.nerf")
    base = dict(ongp.MLP_BASE, hidden_activation=act[hidden],
                density_activation=nerfm.NeRF.DENSITY_ACTIVATION_NAME_TO_FN[density])
    head = dict(ongp.MLP_HEAD, hidden_activation=act[hidden], radiance_activation=ract[radiance], output_dim=rd)
    aabb = [-1.5, -1.5, -1.5, 1.5, 1.5, 1.5]
    field = ngp.NGPradianceField(aabb=aabb, num_dim=3, use_viewdirs=True, contraction_type=ctype,
                                 pos_encoding_config=pos, dir_encoding_config={"degree": 4},
                                 mlp_base_config=base, mlp_head_config=head)
    p = ongp.build_params(rd, seed, pos)
    # a larger table scale than tcnn's 1e-4 init so the encoding dominates the MLP inputs
    p["mlp_base.0.params"] = p["mlp_base.0.params"] * 1e3
    names = [k for k, _ in field.named_parameters()]
    assert set(names) == set(p), (names, list(p))
    field.load_state_dict(dict(p, aabb=field.aabb), strict=True)
    g = torch.Generator().manual_seed(2000 + seed)
    span = 1.8 if contraction == "aabb" else 6.0
    x = (torch.rand(n, 3, generator=g) * 2 * span - span).float()
    d = torch.randn(n, 3, generator=g)
    d = d / d.norm(dim=-1, keepdim=True)
    g_rgb = torch.randn(n, rd, generator=g)
    g_sig = torch.randn(n, 1, generator=g)
    field.zero_grad()
    rgb, sig = field(x, d)
    (rgb * g_rgb).sum().add_((sig * g_sig).sum()).backward()
    out = dict(rgb=rgb.detach().numpy(), sigma=sig.detach().numpy())
    for k, prm in field.named_parameters():
        gr = prm.grad.detach()
        if k == "mlp_base.0.params" and cfg != "small":
            nz = torch.nonzero(gr).flatten()
            out["table_grad_idx"] = nz.numpy()
            out["table_grad_val"] = gr[nz].numpy()
        else:
            out[f"grad:{k}"] = gr.numpy()
    # the default-size table is regenerated in the test from the seed (oracle/ngp.build_params x 1e3)
    extra = dict(table=p["mlp_base.0.params"].numpy()) if cfg == "small" else {}
    mlp_w = {f"param:{k}": v.numpy() for k, v in p.items() if k != "mlp_base.0.params"}
    tag = f"ngp_rd{rd}_{cfg}" + ("" if contraction == "aabb" else f"_{contraction}") + \
        ("" if hidden == "softplus" and radiance == "softplus" else f"_{hidden}_{radiance}") + \
        ("" if density == "shifted_trunc_exp" else f"_{density}")
    save(tag + ".npz", seed=seed, rd=rd, cfg=np.array(cfg), contraction=np.array(contraction), density=np.array(density),
         hidden=np.array(hidden), radiance=np.array(radiance), pos_encoding=np.array(json.dumps(pos)),
         table_sum=np.array(p["mlp_base.0.params"].double().sum().item()), aabb=np.array(aabb, np.float32),
         x=x.numpy(), d=d.numpy(), g_rgb=g_rgb.numpy(), g_sigma=g_sig.numpy(), param_names=np.array(names),
         **out, **extra, **mlp_w)


def _ref_nerf_ngp(rd, seed, res, cfg=None):
    """The reference NeRF with arch "ngp" (models/nerf.py:105-142) in the chair configuration (or
    a step config's aabb / contraction / near / far / cone), oracle/tcnn.py as tcnn.Encoding
    (NGP_SMALL: 8 levels of 2^12 entries), weights from oracle/ngp.build_params(seed) with the
    table x 1e3 -> (nerf, params)."""
    from oracle import ngp as ongp
    from oracle import tcnn as otcnn
    nerfm = _refload.load("models.nerf")
    sys.modules["tinycudann"].Encoding = otcnn.Encoding
    ED = sys.modules["easydict"].EasyDict
    CT = sys.modules["nerfacc"].ContractionType
    c = RENDER_CFG if cfg is None else cfg
    ctype = {"aabb": CT.AABB, "sphere": CT.UN_BOUNDED_SPHERE, "tanh": CT.UN_BOUNDED_TANH}[
        "aabb" if cfg is None else cfg["contraction"]]
    cone = 0.0 if cfg is None else cfg["cone"]
    occ = ED(resolution=res, occ_thre=0.01, ema_decay=0.95, warmup_steps=256, n=16)
    nerf = nerfm.NeRF(c["aabb"], ctype, occ, c["near"], c["far"], c["step"], "parameter", cone, 1e-4, 0.0, 16384,
                      "ngp", ED(NGP_ARCH), 3, rd)
    p = ongp.build_params(rd, seed, dict(NGP_SMALL))
    p["mlp_base.0.params"] = p["mlp_base.0.params"] * 1e3
    rf = nerf.radiance_field
    rf.load_state_dict(dict(p, aabb=rf.aabb), strict=True)
    return nerf, p


def gen_render_ngp(rd=1, seed=25, R=64, sigma_bias_shift=2.0):
    """render_ngp_rd{rd}.npz -- the reference's NeRF.forward with arch "ngp" (models/nerf.py:105-142,
    230-286 -> render_image -> rendering) in the chair configuration: the occupancy-grid update at
    step 0, a training-mode render with its backward, and an eval render -- the flow of gen_render,
    with oracle/tcnn.py as tcnn.Encoding (8 levels of 2^12 entries: the table is stored) and
    oracle/nerfacc.py as nerfacc."""
    from oracle import nerfacc as onerfacc
    c = RENDER_CFG
    nerf, p = _ref_nerf_ngp(rd, seed, c["res"])
    rf = nerf.radiance_field
    out = dict(seed=seed, rd=rd, res=c["res"], step=c["step"], aabb=np.array(c["aabb"]), near=c["near"], far=c["far"],
               sigma_bias_shift=sigma_bias_shift, pos_encoding=np.array(json.dumps(NGP_SMALL)),
               table=p["mlp_base.0.params"].numpy(), **{f"param:{k}": v.numpy() for k, v in p.items()
                                                       if k != "mlp_base.0.params"})
    o, d = _chair_rays(R, 33)
    out.update(rays_o=o.numpy(), rays_d=d.numpy())
    nerf.train()
    torch.manual_seed(100)
    nerf.update_occ_grid(step=0, T_wc_position=o)
    grid = nerf.occupancy_grid
    out.update(occ_u=grid.last_u.numpy(), occs=grid.occs.numpy(), binary=grid.binary.numpy())
    with torch.no_grad():
        rf.mlp_base[1].output_layer.bias[0] += sigma_bias_shift
    r = c["res"]
    cc = (torch.stack(torch.meshgrid(*[torch.arange(r)] * 3, indexing="ij"), -1).float() + 0.5) / r - 0.5
    ball = (cc.norm(dim=-1) < 0.4) & ~((cc[..., 0] > 0.1) & (cc[..., 1].abs() < 0.1))
    grid._binary = ball
    out["binary_render"] = ball.numpy()
    g = torch.Generator().manual_seed(43)
    g_rad = torch.randn(R, rd, generator=g) if rd > 1 else torch.randn(R, generator=g)
    g_op, g_dp = torch.randn(R, generator=g), torch.randn(R, generator=g)
    torch.manual_seed(101)
    rad, op, dp, mspr = nerf(o, d)
    LAST = onerfacc.LAST
    out.update(train_jitter=LAST["jitter"].numpy(), train_kept_ri=LAST["kept"][0].numpy(),
               train_radiance=rad.detach().numpy(), train_opacity=op.detach().numpy(),
               train_depth=dp.detach().numpy(), train_mspr=np.array(mspr), g_rad=g_rad.numpy(), g_op=g_op.numpy(),
               g_dp=g_dp.numpy())
    ((rad * g_rad).sum() + (op * g_op).sum() + (dp * g_dp).sum()).backward()
    for k, prm in rf.named_parameters():
        out[f"grad:{k}"] = prm.grad.detach().numpy()
    out["grad_bkgd_orig"] = nerf.parametrizations.render_bkgd.original.grad.numpy()
    nerf.eval()
    with torch.no_grad():
        rad, op, dp, mspr = nerf(o, d)
    out.update(eval_radiance=rad.numpy(), eval_opacity=op.numpy(), eval_depth=dp.numpy(), eval_mspr=np.array(mspr))
    save(f"render_ngp_rd{rd}.npz", **out)


def gen_render_ngp_cone(rd=1, seed=27, R=64, C=12, sigma_bias_shift=2.0):
    """render_ngp_cone_rd1.npz -- the reference NeRF with the ngp field in configs[3]'s composition
    (07_ziggy_and_fuzz_hdr.yaml:60-75: unbounded-sphere contraction of its aabb, near 0.01 / far 13,
    cone_angle 0.004, a 32^3 grid): the occupancy-grid update at step 0, whose cone branch
    (models/nerf.py:176-193) draws a random camera per cell point (torch.randint, recorded beside
    the cell jitter occ_u) and scales the density by that camera's cone step; then an eval render
    through cone-stepped marching of the updated grid."""
    cfg = _step_cfg(arch="ngp", contraction="sphere", aabb=[0.2, -0.4, 0.0, 3.7, 3.7, 1.8], near=0.01, far=13.0,
                    cone=0.004, res=32)
    nerf, p = _ref_nerf_ngp(rd, seed, cfg["res"], cfg)
    rf = nerf.radiance_field
    a = torch.tensor(cfg["aabb"])
    centre, half = (a[:3] + a[3:]) / 2, (a[3:] - a[:3]) / 2
    g = torch.Generator().manual_seed(seed + 1000)
    v = torch.randn(C, 3, generator=g)
    cams = (centre + v / v.norm(dim=-1, keepdim=True) * float(half.norm()) * 1.3).float()
    out = dict(seed=seed, rd=rd, res=cfg["res"], step=cfg["step"], aabb=np.array(cfg["aabb"], np.float32),
               near=cfg["near"], far=cfg["far"], cone=cfg["cone"], contraction=np.array("sphere"),
               sigma_bias_shift=sigma_bias_shift, pos_encoding=np.array(json.dumps(NGP_SMALL)),
               table=p["mlp_base.0.params"].numpy(), cams=cams.numpy(),
               **{f"param:{k}": v.numpy() for k, v in p.items() if k != "mlp_base.0.params"})
    draws, real_randint = [], torch.randint

    def randint_rec(*ra, **rk):
        r = real_randint(*ra, **rk)
        draws.append(r.clone())
        return r
    nerf.train()
    torch.manual_seed(110)
    torch.randint = randint_rec
    try:
        nerf.update_occ_grid(step=0, T_wc_position=cams)
    finally:
        torch.randint = real_randint
    grid = nerf.occupancy_grid
    assert len(draws) == 1, len(draws)
    out.update(occ_u=grid.last_u.numpy(), occ_randint_0=draws[0].numpy(), occs=grid.occs.numpy(),
               binary=grid.binary.numpy())
    with torch.no_grad():
        rf.mlp_base[1].output_layer.bias[0] += sigma_bias_shift
    idx = torch.randint(0, C, (R,), generator=g)
    o = cams[idx]
    tgt = centre + (torch.rand(R, 3, generator=g) * 2 - 1) * half * 0.6
    d = tgt - o
    d = (d / d.norm(dim=-1, keepdim=True)).float()
    nerf.eval()
    with torch.no_grad():
        rad, op, dp, mspr = nerf(o, d)
    out.update(rays_o=o.numpy(), rays_d=d.numpy(), eval_radiance=rad.numpy(), eval_opacity=op.numpy(),
               eval_depth=dp.numpy(), eval_mspr=np.array(mspr))
    save(f"render_ngp_cone_rd{rd}.npz", **out)


def gen_ngp_all():
    gen_ngp(1, 21, "small")
    gen_ngp(3, 22, "small", "sphere", "relu", "sigmoid")
    gen_ngp(3, 23, "small", "tanh")
    gen_ngp(3, 24, "default", n=256)
    gen_render_ngp(1, 25)
    gen_render_ngp(3, 26)
    gen_step(False, 1, seed=7, tag="step_ngp_nopixbw_rd1.npz", arch="ngp")


def gen_ngp_density():
    gen_ngp(1, 28, "small", density="shifted_softplus")
    gen_ngp(3, 29, "small", "sphere", density="softplus")


def gen_step_ngp():
    gen_step(False, 1, seed=7, tag="step_ngp_nopixbw_rd1.npz", arch="ngp")


def gen_sh():
    """sh_encoder.npz -- the reference's SHEncoder (external/sh_encoder.py:15-193) at every degree
    1..8: out = forward(coords) and d_coords = the autograd gradient of sum(out * g).  Coords: 300
    random unit directions, then 40 non-unit vectors (length 0.3..1.7: the module evaluates its
    polynomials as written), f32."""
    she = _refload.load("external.sh_encoder")
    gen = torch.Generator().manual_seed(31)
    u = torch.randn(340, 3, generator=gen)
    u = u / u.norm(dim=-1, keepdim=True)
    u[300:] *= torch.rand(40, 1, generator=gen) * 1.4 + 0.3
    coords = u.float()
    out = {"coords": coords.numpy()}
    for deg in range(1, 9):
        enc = she.SHEncoder(n_input_dims=3, degree=deg)
        x = coords.clone().requires_grad_(True)
        y = enc(x)
        g = torch.randn(y.shape, generator=gen)
        if y.requires_grad:  # degree 1 is the constant band alone: no graph, a zero gradient
            (y * g).sum().backward()
        out[f"out_{deg}"] = y.detach().numpy()
        out[f"g_{deg}"] = g.numpy()
        out[f"dcoords_{deg}"] = (x.grad if x.grad is not None else torch.zeros_like(x)).numpy()
    save("sh_encoder.npz", **out)


def gen_correction():
    """correction.npz -- the reference's OffsetGammaCorrection (models/offset_gamma_correction.py:4-167)
    on random positive inputs (B 3, C 3, H 4, W 5, R 1) with per-channel and shared parameters:
    forward, jacobian(), param_jacobian()."""
    ogc = _refload.load("models.offset_gamma_correction")
    gen = torch.Generator().manual_seed(41)
    x = torch.rand(3, 3, 4, 5, 1, generator=gen, dtype=torch.float64) * 0.9 + 0.05
    cs = torch.rand(3, 1, 1, 1, 1, generator=gen, dtype=torch.float64) + 0.5
    out = {"x": x.numpy(), "const_scale": cs.numpy()}
    for tag, nS, nG, nO in (("pc", 3, 3, 3), ("shared_gamma", 3, 1, 3), ("scalar", 1, 1, 1)):
        sc = torch.rand(nS, 1, 1, 1, generator=gen, dtype=torch.float64) + 0.5
        ga = torch.rand(nG, 1, 1, 1, generator=gen, dtype=torch.float64) + 0.5
        of = torch.rand(nO, 1, 1, 1, generator=gen, dtype=torch.float64) * 0.1
        m = ogc.OffsetGammaCorrection(cs, sc, ga, of)
        with torch.no_grad():
            out[f"{tag}_scale"], out[f"{tag}_gamma"], out[f"{tag}_offset"] = sc.numpy(), ga.numpy(), of.numpy()
            out[f"{tag}_y"] = m(x).numpy()
            out[f"{tag}_jac"] = m.jacobian(x)[0].numpy()
            for name, j in zip(("scale", "gamma", "offset"), m.param_jacobian(x)[0]):
                out[f"{tag}_pjac_{name}"] = j.numpy()
    save("correction.npz", **out)


def gen_step_ziggy():
    """step_ziggy_rd1.npz -- configs[3]'s model composition (07_ziggy_and_fuzz_hdr.yaml:28-139): the
    ngp arch with the unbounded-sphere contraction of its aabb, near 0.01 / far 13, cone-angle
    marching (0.004), pixel bandwidth with S = 30 samples and every sensor parameter learnable,
    learnable contrast thresholds and refractory period, TV weight 0.1 -- through the reference's
    training_step (16 events, a 32^3 occupancy grid instead of 256^3 so the CPU run finishes)."""
    gen_step(True, 1, seed=9, N=16, S=30, tag="step_ziggy_rd1.npz", arch="ngp", contraction="sphere",
             aabb=[0.2, -0.4, 0.0, 3.7, 3.7, 1.8], near=0.01, far=13.0, cone=0.004, res=32, tv=0.1, pixbw_free=True)


# ----------------------------------------------------------------------------
# raw-event queueing (data/datasets.py:133-187, 190-328): the reference's own per-event loops
QUEUE_CASES = {
    # name: (H, W, N, bayer pattern, timestamps sorted?, seed)
    "small_rggb": (7, 9, 600, "RGGB", True, 1),
    "unsorted_mono": (5, 6, 400, "", False, 2),
    "davis_grbg": (260, 346, 20000, "GRBG", True, 3),
    "hot_pixels_bggr": (2, 3, 30000, "BGGR", True, 4),
}


def synthetic_raw_events(H, W, N, sorted_ts, seed):
    """raw_events.npz-shaped arrays (preprocess_esim.py:314-316, 340-345): position (N,2) uint16
    (x, y), timestamp (N) int64 ns, polarity (N) bool.  Repeated timestamps (zero steps, and
    bursts at one pixel within one timestamp), pixels with a single event, both polarities."""
    g = np.random.default_rng(seed)
    # skewed pixel popularity: some pixels hot, many cold
    wts = g.pareto(1.2, size=H * W) + 1e-3
    wts[g.random(H * W) < 0.3] = 0.0  # never fire
    wts /= wts.sum()
    pix = g.choice(H * W, size=N, p=wts)
    steps = g.integers(0, 4, size=N) * g.integers(1, 500, size=N)  # ~1/4 zero steps
    ts = 1_000_000 + np.cumsum(steps).astype(np.int64)
    # bursts: an event repeated at its own pixel with its own timestamp
    rep = g.random(N) < 0.05
    pix[1:][rep[1:]] = pix[:-1][rep[1:]]
    ts[1:][rep[1:]] = ts[:-1][rep[1:]]
    if not sorted_ts:
        ts = ts[g.permutation(N)]
    pos = np.stack([pix % W, pix // W], axis=1).astype(np.uint16)
    pol = g.random(N) < 0.5
    return pos, ts, pol


def gen_queue():
    """queue_<case>.npz: Event.queue_raw_events -> colorize_events -> undistort_events (no
    distortion parameters: the f32 cast only) and Event.extract_max_refractory_period, the
    reference's classmethods run as-is on a temporary dataset directory."""
    ds = _refload.load("data.datasets")
    for name, (H, W, N, bayer, sorted_ts, seed) in QUEUE_CASES.items():
        pos, ts, pol = synthetic_raw_events(H, W, N, sorted_ts, seed)
        d = tempfile.mkdtemp(prefix="den_raw_")
        np.savez(os.path.join(d, "raw_events.npz"), position=pos, timestamp=ts, polarity=pol)
        cal = dict(img_height=np.array(H, dtype=np.uint16), img_width=np.array(W, dtype=np.uint16),
                   bayer_pattern=np.array(bayer), distortion_model=np.array("plumb_bob"),
                   distortion_params=np.zeros(0, dtype=np.float32),
                   intrinsics=np.array([[200.0, 0, W / 2], [0, 200.0, H / 2], [0, 0, 1]], dtype=np.float32))
        np.savez(os.path.join(d, "camera_calibration.npz"), **cal)
        calib = np.load(os.path.join(d, "camera_calibration.npz"))
        q = ds.Event.queue_raw_events(d, calib)
        queued = {k: v.clone() for k, v in q.items()}
        col = ds.Event.colorize_events(q, calib)
        und = ds.Event.undistort_events(col, calib)
        mx = ds.Event.extract_max_refractory_period(np.load(os.path.join(d, "raw_events.npz")), calib)
        out = dict(raw_position=pos, raw_timestamp=ts, raw_polarity=pol, img_height=H, img_width=W,
                   bayer_pattern=np.array(bayer), max_refractory_period=mx.numpy(),
                   max_refractory_period_dtype=np.array(str(mx.dtype)),
                   final_position=und.position.numpy(), final_position_dtype=np.array(str(und.position.dtype)))
        for k, v in queued.items():
            out["q_" + k] = v.numpy()
        if "channel_idx" in col:
            out["channel_idx"] = col.channel_idx.numpy()
        save(f"queue_{name}.npz", **out)
    # no interval anywhere: every pixel fires once, or repeats its own timestamp -> inf, nothing queued
    H, W = 4, 4
    pos = np.array([[0, 0], [1, 0], [1, 0], [2, 3], [3, 3], [3, 3], [3, 3]], dtype=np.uint16)
    ts = np.array([5, 9, 9, 11, 20, 20, 20], dtype=np.int64)
    pol = np.array([1, 0, 1, 1, 0, 0, 1], dtype=bool)
    d = tempfile.mkdtemp(prefix="den_raw_")
    np.savez(os.path.join(d, "raw_events.npz"), position=pos, timestamp=ts, polarity=pol)
    np.savez(os.path.join(d, "camera_calibration.npz"), img_height=np.array(H, dtype=np.uint16),
             img_width=np.array(W, dtype=np.uint16), bayer_pattern=np.array(""))
    calib = np.load(os.path.join(d, "camera_calibration.npz"))
    q = ds.Event.queue_raw_events(d, calib)
    mx = ds.Event.extract_max_refractory_period(np.load(os.path.join(d, "raw_events.npz")), calib)
    save("queue_no_interval.npz", raw_position=pos, raw_timestamp=ts, raw_polarity=pol, img_height=H, img_width=W,
         q_count=np.array(len(q.position)), max_refractory_period=mx.numpy(),
         max_refractory_period_dtype=np.array(str(mx.dtype)))


# ----------------------------------------------------------------------------
# evaluation views (data/datasets.py:376-712 PosedImage) and the evaluation loop
# (models/deblur_e_nerf.py:588-1053), run through the reference's own code
from pngenc import bgr as _bgr, encode_png  # noqa: E402


IMREAD_TRUTH = {}


def install_cv2():
    """cv2 stand-in for the reference's PosedImage / evaluation_epoch_end: imread returns the exact
    samples the fixture wrote to that path in OpenCV's conventions (BGR / BGRA order, grey + alpha
    expanded to BGRA, the file's sample type); cvtColor restates COLOR_BGR2RGB / COLOR_RGB2BGR (the
    channel order reversed) and COLOR_BGR2GRAY on float32 as OpenCV 4.5.2's SIMD path computes it,
    fma(r, 0.299f, fma(g, 0.587f, b * 0.114f)) (evaluated exactly in f64, rounded per operation);
    imwrite records the arrays it is given."""
    cv2 = sys.modules["cv2"]
    cv2.IMREAD_UNCHANGED, cv2.COLOR_BGR2RGB, cv2.COLOR_RGB2BGR, cv2.COLOR_BGR2GRAY = -1, 4, 4, 6
    cv2.written = {}

    def imread(path, flags):
        assert flags == -1
        return IMREAD_TRUTH[os.path.realpath(path)].copy()

    def cvtColor(img, code):
        if code == 4:
            assert img.ndim == 3 and img.shape[2] == 3
            return np.ascontiguousarray(img[..., ::-1])
        assert code == 6 and img.dtype == np.float32
        c = [np.float64(np.float32(v)) for v in (0.114, 0.587, 0.299)]
        b, g, r = (img[..., k].astype(np.float64) for k in range(3))
        t = (b * c[0]).astype(np.float32).astype(np.float64)
        t = (g * c[1] + t).astype(np.float32).astype(np.float64)
        return (r * c[2] + t).astype(np.float32)

    def imwrite(path, img):
        cv2.written[os.path.basename(path)] = np.array(img)
        return True

    cv2.imread, cv2.cvtColor, cv2.imwrite = imread, cvtColor, imwrite
    return cv2


def _view_poses(n, seed, radius=4.03):
    """n camera-to-world matrices in the OpenGL convention (x right, y up, z back) looking at the
    origin from radius ~4 (the layout of the synthetic chair views)."""
    g = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        v = g.normal(size=3)
        c = v / np.linalg.norm(v) * radius
        z = c / np.linalg.norm(c)           # back = away from the origin
        x = np.cross([0.0, 0.0, 1.0], z)
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        T = np.eye(4)
        T[:3, 0], T[:3, 1], T[:3, 2], T[:3, 3] = x, y, z, c
        out.append(T)
    return out


POSED_CASES = {
    # name: bayer, renderer (None | display | linear), sample depth, channels, file kind, intrinsics
    # source, per-frame exposure / gain, bit_depth key, views folder one level up, runs (stage, perm
    # seed, alpha over white)
    "mono_display_rgba8": dict(bayer="", renderer="display", depth=8, C=4, kind="png", fov=True, expo=False,
                               bit_depth=None, up=False, runs=[("val", None, True), ("val", 9, True),
                                                               ("test", None, False)]),
    "rggb_real_rgb8": dict(bayer="RGGB", renderer=None, depth=8, C=3, kind="png", fov=False, expo=True,
                           bit_depth=None, up=True, runs=[("train", None, False), ("train", 3, False)]),
    "mono_real_gray16_bd10": dict(bayer="", renderer=None, depth=16, C=1, kind="png", fov=True, expo=True,
                                  bit_depth=10, up=False, runs=[("val", None, False)]),
    "rggb_display_rgba16": dict(bayer="BGGR", renderer="display", depth=16, C=4, kind="png", fov=True, expo=False,
                                bit_depth=None, up=False, runs=[("val", None, True), ("val", None, False)]),
    "mono_display_ga16": dict(bayer="", renderer="display", depth=16, C=2, kind="png", fov=True, expo=False,
                              bit_depth=None, up=False, runs=[("val", None, True)]),
    "mono_real_rgb8": dict(bayer="", renderer=None, depth=8, C=3, kind="pil", fov=True, expo=False,
                           bit_depth=None, up=False, runs=[("val", 1, False)]),
    "mono_linear_npy": dict(bayer="", renderer="linear", depth=32, C=4, kind="npy", fov=True, expo=False,
                            bit_depth=None, up=False, runs=[("val", None, True), ("val", None, False)]),
    "rggb_linear_npy": dict(bayer="RGGB", renderer="linear", depth=32, C=3, kind="npy", fov=False, expo=False,
                            bit_depth=None, up=False, runs=[("val", None, False)]),
}


def _case_samples(c, n, H, W, g):
    """n images of samples for a case: smooth gradients + noise in the file's range."""
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    imgs = []
    for k in range(n):
        chans = []
        for ch in range(c["C"]):
            base = 0.5 + 0.4 * np.sin(3 * xx + 2 * yy * (ch + 1) + k) + 0.05 * g.normal(size=(H, W))
            if ch == 3 or (c["C"] == 2 and ch == 1):  # alpha: opaque centre, transparent corners
                base = np.clip(1.6 - 2.5 * np.hypot(xx - 0.5, yy - 0.5), 0, 1)
            chans.append(np.clip(base, 0, 1))
        a = np.stack(chans, -1) if c["C"] > 1 else chans[0]
        if c["kind"] == "npy":
            a = a.astype(np.float32)
            if c["C"] == 4:  # premultiplied alpha (linear renders)
                a[..., :3] *= a[..., 3:4]
            imgs.append(a)
            continue
        top = (2 ** c["bit_depth"] - 1) if c["bit_depth"] else (2 ** c["depth"] - 1)
        imgs.append(np.round(a * top).astype(np.uint16 if c["depth"] == 16 else np.uint8))
    return imgs


def write_posed_case(name, c, root, seed=5, H=20, W=24):
    """A dataset directory for a PosedImage case: camera_calibration.npz, [renderer_params.npz],
    views/transforms_{stage}.json and the image files (PNG by the encoder above or by PIL, or .npy).
    Registers what cv2.imread returns for each image.  -> {relative path: file bytes}."""
    from PIL import Image
    g = np.random.default_rng(seed)
    cal = dict(bayer_pattern=np.array(c["bayer"]), intrinsics=np.array([[30.0, 0, 12], [0, 30.0, 10], [0, 0, 1]],
                                                                      dtype=np.float32),
               img_height=np.array(H), img_width=np.array(W))
    np.savez(os.path.join(root, "camera_calibration.npz"), **cal)
    if c["renderer"] is not None:
        np.savez(os.path.join(root, "renderer_params.npz"), interm_color_space=np.array(c["renderer"]),
                 log_eps=np.array(0.001))
    views = os.path.join(root, "..", "views") if c["up"] else os.path.join(root, "views")
    os.makedirs(views, exist_ok=True)
    stages = sorted({r[0] for r in c["runs"]})
    for si, stage in enumerate(stages):
        os.makedirs(os.path.join(views, stage), exist_ok=True)
        n = 3 + si
        imgs = _case_samples(c, n, H, W, g)
        frames = []
        for k, (img, T) in enumerate(zip(imgs, _view_poses(n, seed + 17 * si))):
            rel = f"./{stage}/r_{k}" if k != 1 else f"./{stage}/view_long_name{k}"
            path = os.path.join(views, rel[2:]) + {"png": ".png", "pil": ".png", "npy": ".npy"}[c["kind"]]
            if c["kind"] == "npy":
                np.save(path, _bgr(img))   # float renders stored as OpenCV hands them over (BGR[A])
            elif c["kind"] == "pil":
                Image.fromarray(img).save(path)
            else:
                with open(path, "wb") as f:
                    f.write(encode_png(img, c["depth"]))
            IMREAD_TRUTH[os.path.realpath(path)] = _bgr(img) if c["kind"] != "npy" else _bgr(img)
            fr = {"file_path": rel, "transform_matrix": T.tolist()}
            if c["expo"]:
                fr["exposure_time"] = int(g.integers(5_000_000, 20_000_000))
                fr["gain"] = float(g.uniform(0.5, 4.0))
            frames.append(fr)
        tf = {"frames": frames}
        if c["fov"]:
            tf["camera_angle_x"] = 0.6911112070083618
        else:
            tf["intrinsics"] = [[28.0, 0.0, 11.5], [0.0, 29.0, 9.5], [0.0, 0.0, 1.0]]
        if c["bit_depth"]:
            tf["bit_depth"] = c["bit_depth"]
        with open(os.path.join(views, f"transforms_{stage}.json"), "w") as f:
            json.dump(tf, f, indent=2)
    files = {}
    base = os.path.dirname(root) if c["up"] else root
    for dirpath, _, names in os.walk(base):
        for nm in names:
            full = os.path.join(dirpath, nm)
            with open(full, "rb") as f:
                files[os.path.relpath(full, base)] = f.read()
    return files


def gen_posed():
    """posed_<case>.npz -- the reference's PosedImage (data/datasets.py:376-712) run as-is on the
    synthetic view directories of POSED_CASES (cv2 as install_cv2 states it): every output of each
    (stage, permutation seed, alpha over white) run.  The directory's files are stored as bytes
    (``file:<relative path>``) so the tests rebuild it; ``root`` names the dataset directory among them."""
    ds = _refload.load("data.datasets")
    install_cv2()
    for name, c in POSED_CASES.items():
        top = tempfile.mkdtemp(prefix="den_posed_")
        root = os.path.join(top, "seq") if c["up"] else top
        os.makedirs(root, exist_ok=True)
        files = write_posed_case(name, c, root)
        out = {f"file:{k}": np.frombuffer(v, dtype=np.uint8) for k, v in files.items()}
        out["root"] = np.array("seq" if c["up"] else ".")
        out["n_runs"] = np.array(len(c["runs"]))
        for i, (stage, perm, alpha) in enumerate(c["runs"]):
            pi = ds.PosedImage(root, stage, perm, alpha)
            p = f"run{i}:"
            out[p + "stage"], out[p + "perm"], out[p + "alpha"] = np.array(stage), np.array(-1 if perm is None else perm), \
                np.array(alpha)
            for k, v in pi.posed_imgs.items():
                out[p + k] = v.numpy()
                out[p + k + "_dtype"] = np.array(str(v.dtype))
            out[p + "min_normalized_pixel_value"] = np.array(float(pi.min_normalized_pixel_value))
            out[p + "max_normalized_pixel_value"] = np.array(float(pi.max_normalized_pixel_value))
        save(f"posed_{name}.npz", **out)


class _ImgLogger:
    """What evaluation_epoch_end uses of a TensorBoard logger: experiment.add_image."""

    def __init__(self):
        self.images = {}
        self.experiment = self

    def add_image(self, tag, img, global_step=None):
        self.images[tag] = img.detach().cpu().numpy()


def gen_eval_epoch(rd=1, seed=6, H=20, W=24, black_level_offset=True, algo="lm", tag=None, sigma_bias_shift=2.0,
                   rgb_weight_scale=30.0):
    """eval_epoch_*.npz -- the reference's validation loop: PosedImage views (8-bit PNG: RGB for the
    monochrome sensor, RGBA alpha-composited over white for the Bayer one), the DataModule's permuted order and batches of one,
    DeblurENeRF.validation_step (render_pixels over the view's pixel grid at its pose, eval mode)
    and validation_epoch_end (the gather; the affine log-intensity correction; with
    ``black_level_offset`` the OffsetGammaCorrection refinement by the reference's own
    external/optimizer.py on oracle/pypose.py; Metric (l1, psnr, ssim via oracle/metrics.py); the
    correction-error CSV, the logged images and the saved 8-bit predictions) -- twice, the second
    evaluation warm-started from the first's converged correction.  The targets are the reference
    model's own renders under a known gamma / scale / black level, quantised; the radiance output
    layer's weights are scaled by ``rgb_weight_scale`` so the renders span a wide intensity range (a
    random-init field renders an almost flat image, on which the correction's scale and gamma
    columns are collinear and its refinement ill-conditioned)."""
    cfg = _step_cfg(rd=rd)
    cal, poses = synthetic_dataset_arrays(rd)
    d = tempfile.mkdtemp(prefix="den_evalep_")
    write_dataset(d, cal, poses)
    m = ref_deblur_step_module(d, seed, cfg)
    with torch.no_grad():
        m.nerf.radiance_field.mlp.sigma_layer.output_layer.bias.add_(sigma_bias_shift)
        m.nerf.radiance_field.mlp.rgb_layer.output_layer.weight.mul_(rgb_weight_scale)
    torch.manual_seed(300)
    m.nerf.update_occ_grid(step=0, T_wc_position=m.trajectory.T_wc_position)
    grid = m.nerf.occupancy_grid
    m.eval()
    ds = _refload.load("data.datasets")
    _refload.load("external.optimizer")  # deblur_e_nerf.py reaches it as external.optimizer (pypose stand-in)
    install_cv2()
    ED = sys.modules["easydict"].EasyDict
    # the views: renders of the reference model at 3 poses, mapped through a gamma / scale / black level,
    # quantised to 8 bits, RGBA with an opaque alpha (display renders)
    views = os.path.join(d, "views")
    os.makedirs(os.path.join(views, "val"))
    fov = 0.9
    f = (W / 2) / np.tan(fov / 2)
    K = torch.tensor([[f, 0, W / 2 - 0.5], [0, f, H / 2 - 0.5], [0, 0, 1]], dtype=torch.float32)
    pix = torch.stack(torch.meshgrid(torch.arange(W), torch.arange(H), indexing="xy"), dim=2).float()
    frames = []
    g = np.random.default_rng(seed)
    for k, T in enumerate(_view_poses(3, seed + 1)):
        rot = torch.tensor(T[:3, :3] @ np.diag([1.0, -1.0, -1.0]), dtype=torch.float32)
        pos = torch.tensor(T[:3, 3], dtype=torch.float32)
        with torch.no_grad():
            img, _, _, _, _ = m.render_pixels(torch.linalg.inv(K), pix, pos.view(1, 1, 3).expand(H, W, -1),
                                              rot.view(1, 1, 3, 3).expand(H, W, -1, -1))
        lin = img.numpy().astype(np.float64)
        print(f"[eval_epoch rd={rd}] view {k}: render range {lin.min():.4f}..{lin.max():.4f}")
        lin = 0.9 * np.power(lin / lin.max(), 0.8) + 0.03 + 0.01 * g.normal(size=lin.shape)
        q = np.round(np.clip(lin, 0, 1) * 255).astype(np.uint8)
        # a monochrome sensor gets RGB files (converted to grey; the reference converts only 3-channel
        # views, datasets.py:639-644), a Bayer sensor RGBA ones alpha-composited over white
        rgb = np.stack([q] * 3, -1) if rd == 1 else q.transpose(1, 2, 0)
        if rd == 3:
            alpha = np.full(rgb.shape[:2] + (1,), 255, np.uint8)
            alpha[:3, :4] = 128
            rgb = np.concatenate([rgb, alpha], -1)
        path = os.path.join(views, "val", f"r_{k}.png")
        with open(path, "wb") as fh:
            fh.write(encode_png(rgb, 8))
        IMREAD_TRUTH[os.path.realpath(path)] = _bgr(rgb)
        frames.append({"file_path": f"./val/r_{k}", "transform_matrix": T.tolist()})
    with open(os.path.join(views, "transforms_val.json"), "w") as fh:
        json.dump({"camera_angle_x": fov, "frames": frames}, fh)
    np.savez(os.path.join(d, "renderer_params.npz"), interm_color_space=np.array("display"), log_eps=np.array(0.001))
    # DeblurENeRF.__init__'s evaluation state (deblur_e_nerf.py:96-127, 164-197)
    vp = ds.PosedImage(d, "val", permutation_seed=None)
    m.val_min_normalized_pixel_value = vp.min_normalized_pixel_value
    m.val_max_normalized_pixel_value = vp.max_normalized_pixel_value
    m.register_buffer("val_intrinsics_inv", vp.posed_imgs.intrinsics.inverse(), persistent=False)
    m.register_buffer("val_img_pixel_pos", torch.stack(torch.meshgrid(torch.arange(W), torch.arange(H), indexing="xy"),
                                                       dim=2).to(torch.get_default_dtype()), persistent=False)
    m.correction = ED(per_channel_log_it_scale=False, black_level_offset=black_level_offset,
                      optimizer=ED(algo=algo, max_steps=10, lm=ED(radius=1.0e6)))
    rdim = 3 if m.has_bayer_filter else 1
    if black_level_offset:
        m.init_correction_scale = torch.ones((rdim, 1, 1, 1), dtype=torch.float64)
        m.init_correction_offset = torch.zeros((rdim, 1, 1, 1), dtype=torch.float64)
        m.init_correction_gamma = torch.ones((rdim if not m.has_bayer_filter else 1, 1, 1, 1), dtype=torch.float64)
    m.metric = _refload.load("loss_metric.metric").Metric("alex")
    m.eval_save_pred_intensity_img = True
    logdir = tempfile.mkdtemp(prefix="den_evallog_")
    m.trainer = types.SimpleNamespace(log_dir=logdir, is_global_zero=True, sanity_checking=False,
                                      accumulate_grad_batches=1)
    m.logger = _ImgLogger()
    m.device = torch.device("cpu")
    m.all_gather = lambda t: t  # PL single-device all_gather
    logged = {}
    m.log = lambda name, value, **kw: logged.__setitem__(name, value)
    # the DataModule's val set: PosedImage with the config's permutation seed and alpha over white
    val = ds.PosedImage(d, "val", 9, rd == 3)
    out = dict(rd=rd, seed=seed, N=0, S=8, pixbw=False, res=cfg["res"], sigma_bias_shift=sigma_bias_shift,
               rgb_weight_scale=rgb_weight_scale, occ_u=grid.last_u.numpy(), occs=grid.occs.numpy(), black_level_offset=black_level_offset,
               algo=np.array(algo), eval_perm_seed=9, alpha_over_white_bg=rd == 3,
               **{f"cal:{k}": v for k, v in cal.items()}, **{f"pose:{k}": v for k, v in poses.items()})
    base = d
    for dirpath, _, names in os.walk(os.path.join(d, "views")):
        for nm in names:
            full = os.path.join(dirpath, nm)
            with open(full, "rb") as fh:
                out["file:" + os.path.relpath(full, base)] = np.frombuffer(fh.read(), dtype=np.uint8)
    with open(os.path.join(d, "renderer_params.npz"), "rb") as fh:
        out["file:renderer_params.npz"] = np.frombuffer(fh.read(), dtype=np.uint8)
    for ev in range(2):
        m.current_epoch = ev
        logged.clear()
        sys.modules["cv2"].written.clear()
        m.logger.images.clear()
        outputs = []
        with torch.no_grad():
            for i in range(len(val)):
                batch = torch.utils.data.default_collate([val[i]])
                outputs.append(m.validation_step(batch, i))
        p = f"ev{ev}:"
        out[p + "pred"] = torch.stack([o["pred_intensity_img"] for o in outputs]).numpy()
        with torch.no_grad():
            m.validation_epoch_end(outputs)
        for k, v in logged.items():
            out[p + "log:" + k] = np.array(float(v))
        if black_level_offset:
            out[p + "init_scale"] = m.init_correction_scale.numpy()
            out[p + "init_gamma"] = m.init_correction_gamma.numpy()
            out[p + "init_offset"] = m.init_correction_offset.numpy()
            out[p + "errors"] = np.loadtxt(os.path.join(logdir, "correction-errors", f"{ev}.csv"), ndmin=1)
        for k, v in m.logger.images.items():
            out[p + "image:" + k] = v
        for k, v in sys.modules["cv2"].written.items():
            out[p + "saved:" + k] = v
    save(tag or f"eval_epoch_rd{rd}.npz", **out)


def gen_eval_epoch_all():
    gen_eval_epoch(1, seed=6)
    gen_eval_epoch(3, seed=8, algo="gn", tag="eval_epoch_rd3_gn.npz")
    gen_eval_epoch(1, seed=10, black_level_offset=False, tag="eval_epoch_rd1_affine.npz")


if __name__ == "__main__" and len(sys.argv) > 1:
    torch.set_num_threads(8)
    for name in sys.argv[1:]:
        globals()["gen_" + name]()
elif __name__ == "__main__":
    torch.set_num_threads(8)
    gen_mlp(3, seed=0)
    gen_mlp(1, seed=1)
    gen_mlp_unbounded()
    gen_foh()
    gen_pixbw(16, EDS, "eds")
    gen_pixbw(30, EDS, "eds")
    gen_pixbw(16, PERTURBED, "pert")
    gen_loss()
    gen_ct()
    gen_events()
    gen_rays()
    gen_render(1, 4)
    gen_render(3, 5)
    gen_traj()
    gen_step(False, 1)
    gen_step(True, 1)
    gen_ngp_all()
    gen_queue()
    gen_posed()
    gen_eval_epoch_all()
