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
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
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
def gen_mlp(rd, seed):
    mlp = _refload.load("external.mlp")
    ngp = _refload.load("external.ngp")
    ContractionType = sys.modules["nerfacc"].ContractionType
    torch.manual_seed(seed)
    field = mlp.VanillaNeRFRadianceField(
        aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], net_depth=8, net_width=256,
        skip_layer=4, net_depth_condition=1, net_width_condition=128, num_dim=3,
        contraction_type=ContractionType.AABB, radiance_dim=rd,
        hidden_activation=torch.nn.Softplus(beta=100),
        density_activation=ngp.shifted_trunc_exp,
        radiance_activation=torch.nn.Softplus(beta=1),
        pos_encoder_max_deg=10, view_encoder_max_deg=4, weight_norm=False)
    g = torch.Generator().manual_seed(1000 + seed)
    n = 512
    # positions: mostly inside the AABB, some outside (selector = 0)
    x = (torch.rand(n, 3, generator=g) * 3.6 - 1.8).float()
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
    save(f"mlp_rd{rd}.npz", seed=seed, x=x.numpy(), d=d.numpy(), g_rgb=g_rgb.numpy(),
         g_sigma=g_sig.numpy(), param_names=np.array(names), **out, **wsum)


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
    for efn_diff, efn_tv in (("huber", "l1"), ("l1", "huber"), ("mse", "mse")):
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


if __name__ == "__main__" and len(sys.argv) > 1:
    torch.set_num_threads(8)
    for name in sys.argv[1:]:
        globals()["gen_" + name]()
elif __name__ == "__main__":
    torch.set_num_threads(8)
    gen_mlp(3, seed=0)
    gen_mlp(1, seed=1)
    gen_foh()
    gen_pixbw(16, EDS, "eds")
    gen_pixbw(30, EDS, "eds")
    gen_pixbw(16, PERTURBED, "pert")
    gen_loss()
    gen_ct()
    gen_events()
    gen_rays()
