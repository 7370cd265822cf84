"""Native training step of the render + event-measurement hot path.

``TrainStep`` is one ``DeblurENeRF.training_step`` + DDP gradient all-reduce +
``Adam.step`` (deblur_e_nerf.py:396-586, 1055-1112; scripts/run.py:84-100)
for the synthetic configuration of BASELINE.json (chair, pixel-bandwidth model
off, mlp arch), with every array operation in libden.so:

  [den_event_prep -> den_pixel_rays, when fed raw events (load_events)]
  -> den_event_target (when fed prepared rays, load_batch) -> den_render_fwd (4 render groups x N events in ONE launch)
  -> den_event_step_fwd/bwd (log-intensity, Huber diff + L1 TV losses and their
  gradient) -> den_render_bwd (compositing adjoint, MLP backward, split-K weight
  gradients) -> RCCL all-reduce of one flat f32 gradient buffer (ranks > 1)
  -> den_adam_step (L2 weight decay 1e-6 on the MLP) -> den_pack_weights.

The only PyTorch arithmetic is the softplus parametrisation of the rd-element
render background (a scalar parameter transform, as utils/modules.py keeps).
"""
import ctypes
import math

import numpy as np
import torch
import torch.distributed as dist

from . import _native as nat
from .external import mlp, ngp

ERR = nat.ERROR_FNS


def allreduce_mean(buf):
    """DDP gradient semantics (scripts/run.py:84-89): the mean over ranks of the
    per-rank gradients, one collective on one flat buffer (RCCL on the GPU box,
    gloo in the CPU tests).  No-op for a single process."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        buf.div_(dist.get_world_size())
    return buf


class TrainStep:
    def __init__(self, n_events, n_samples=128, radiance_dim=1, mode="bf16", seed=0, device="cuda",
                 aabb=(-1.5, -1.5, -1.5, 1.5, 1.5, 1.5), near=1.43, far=6.63, lr=0.01, weight_decay=1e-6,
                 loss_weight=(1.0, 1e-3), error_fn=("huber", "l1"), min_modeled_intensity=1e-3,
                 mean_contrast_threshold=0.25, alpha_over_white_bg=True, contrast_thresholds=None,
                 refractory_period=0.0):
        self.N, self.S, self.rd, self.mode = n_events, n_samples, radiance_dim, nat.mode_id(mode)
        self.dev = torch.device(device)
        self.R = 4 * n_events
        torch.manual_seed(seed)
        field = mlp.VanillaNeRFRadianceField(
            list(aabb), radiance_dim=radiance_dim, hidden_activation=torch.nn.Softplus(beta=100),
            density_activation=ngp.shifted_trunc_exp, radiance_activation=torch.nn.Softplus(beta=1),
            mode=mode)
        self.P = nat.param_count(radiance_dim)
        self.flat = field.flat_params.detach().to(self.dev).contiguous()
        assert self.flat.numel() == self.P
        # one flat gradient buffer [MLP params | render bkgd] -> one collective per step
        self.gbuf = torch.zeros(self.P + radiance_dim, device=self.dev)
        self.grad = self.gbuf[: self.P]
        self.grad_bkgd = self.gbuf[self.P:]
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.has_bkgd = bool(alpha_over_white_bg)
        # nerf.py:219-228: Parameter(ones(rd)) under a softplus parametrisation
        self.bkgd_orig = torch.full((radiance_dim,), math.log(math.expm1(1.0)), device=self.dev)
        self.bm = torch.zeros_like(self.bkgd_orig)
        self.bv = torch.zeros_like(self.bkgd_orig)
        self.t = 0
        self.lr, self.wd = lr, weight_decay
        self.wl, self.fn = loss_weight, error_fn
        self.min_int = min_modeled_intensity
        self.c = torch.tensor([mean_contrast_threshold], device=self.dev)
        # post-parametrisation C+, C- and tau_r (frozen in the synthetic configuration,
        # configs/train/synthetic.yaml:29-40); C+ = C- = mean unless given
        cp = contrast_thresholds or (mean_contrast_threshold, mean_contrast_threshold)
        self.ct = torch.tensor(cp, dtype=torch.float32, device=self.dev)
        self.tau = torch.tensor([refractory_period], dtype=torch.float64, device=self.dev)
        self.raw = False
        self.cfg = dict(mode=self.mode, rd=radiance_dim, aabb=list(aabb), near=near, far=far)
        self.packed = nat.PackedWeights(self.mode, radiance_dim, self.dev)
        self.packed.pack(self.flat)
        self.desc = nat._desc(self.cfg, self.R, n_samples, True, self.has_bkgd)
        self.ws = torch.empty(nat.render_workspace_bytes(self.desc), dtype=torch.uint8, device=self.dev)
        self.rgb = torch.empty(self.R, radiance_dim, device=self.dev)
        self.opacity = torch.empty(self.R, device=self.dev)
        self.depth = torch.empty(self.R, device=self.dev)
        self.d_rgb = torch.empty_like(self.rgb)
        self.ev_ws = torch.empty(nat.lib().den_event_step_workspace_bytes(n_events) // 4 + 1, device=self.dev)
        self.loss = torch.zeros(4, device=self.dev)
        self.target = torch.empty(n_events, device=self.dev)

    # ---------------------------------------------------------------- batch
    def load_batch(self, rays_o, rays_d, jitter, lid, end_ts, start_ts, ts_diff, channel=None):
        """rays_* : (4N, 3) for groups [diff start, diff end, tv start, tv end];
        lid (N) f32 measured log-intensity change; end_ts (N) i64; start_ts, ts_diff (N) f64."""
        d = self.dev
        self.rays_o = rays_o.to(d, torch.float32).contiguous()
        self.rays_d = rays_d.to(d, torch.float32).contiguous()
        self.jitter = jitter.to(d, torch.float32).contiguous()
        self.lid = lid.to(d, torch.float32).contiguous()
        self.end_ts = end_ts.to(d, torch.int64).contiguous()
        self.start_ts = start_ts.to(d, torch.float64).contiguous()
        self.ts_diff = ts_diff.to(d, torch.float64).contiguous()
        self.channel = None if channel is None else channel.to(d, torch.int64).contiguous()

    def load_events(self, num_pos, num_neg, end_ts, start_ts, normalized, position, T_wc_position,
                    T_wc_orientation, intrinsics_inverse, jitter, channel=None):
        """Raw events as the datamodule hands them to training_step
        (deblur_e_nerf.py:396-455): num_pos, num_neg, end_ts, start_ts (N) i64,
        normalized (4,N) f64 [ts_diff, diff_start_ts, ts_subdiff, subdiff_start_ts],
        pixel position (N,2) f32, and the camera poses at the 4 render timestamps
        (4,N,3) / (4,N,3,3) f32 (the trajectory's output), K^-1 (3,3), per-ray
        sampler jitter (4N).  Every step then derives the event corrections,
        timestamps, target and rays on the device (den_event_prep, den_pixel_rays)."""
        d = self.dev
        i64 = lambda t: t.to(d, torch.int64).contiguous()
        f32 = lambda t: t.to(d, torch.float32).contiguous()
        self.ev = dict(num_pos=i64(num_pos), num_neg=i64(num_neg), end_ts=i64(end_ts), start_ts=i64(start_ts))
        self.norm = normalized.to(d, torch.float64).contiguous()
        self.position, self.T_pos, self.T_rot = f32(position), f32(T_wc_position), f32(T_wc_orientation)
        self.K_inv = f32(intrinsics_inverse)
        self.jitter = f32(jitter)
        self.end_ts = self.ev["end_ts"]
        self.channel = None if channel is None else i64(channel)
        N = self.N
        self.lid = torch.empty(N, device=d)
        self.start_ts = torch.empty(N, dtype=torch.float64, device=d)
        self.render_ts = torch.empty(4, N, dtype=torch.float64, device=d)
        self.ts_diff = torch.empty(N, dtype=torch.float64, device=d)
        self.ts_subdiff = torch.empty(N, dtype=torch.float64, device=d)
        self.rays_o = torch.empty(4 * N, 3, device=d)
        self.rays_d = torch.empty(4 * N, 3, device=d)
        self.raw = True

    # ---------------------------------------------------------------- phases
    def prepare(self):
        """Raw events -> lid, refractory-shifted start, supervision timestamps,
        diff target (den_event_prep) and the 4N rays (den_pixel_rays)."""
        L, st = nat.lib(), nat._stream(self.dev)
        e = self.ev
        nat._check(L.den_event_prep(self.N, 1, 1, nat._ptr(e["num_pos"]), nat._ptr(e["num_neg"]),
                                    nat._ptr(e["end_ts"]), nat._ptr(e["start_ts"]), nat._ptr(self.norm),
                                    nat._ptr(self.ct), nat._ptr(self.tau), nat._ptr(self.c), nat._ptr(self.lid),
                                    nat._ptr(self.start_ts), nat._ptr(self.render_ts), nat._ptr(self.ts_diff),
                                    nat._ptr(self.ts_subdiff), nat._ptr(self.target), st))
        nat._check(L.den_pixel_rays(4, self.N, nat._ptr(self.K_inv), nat._ptr(self.position), nat._ptr(self.T_pos),
                                    nat._ptr(self.T_rot), nat._ptr(self.rays_o), nat._ptr(self.rays_d), st))

    def forward(self):
        L, st = nat.lib(), nat._stream(self.dev)
        self.bkgd = torch.nn.functional.softplus(self.bkgd_orig) if self.has_bkgd else None
        if self.raw:
            self.prepare()
        else:
            nat._check(L.den_event_target(self.N, nat._ptr(self.ts_diff), nat._ptr(self.lid), nat._ptr(self.end_ts),
                                          nat._ptr(self.start_ts), nat._ptr(self.c), nat._ptr(self.target), st))
        self.io = nat.RenderIO(nat._ptr(self.rays_o), nat._ptr(self.rays_d), nat._ptr(self.jitter),
                               nat._ptr(self.packed.fwd), nat._ptr(self.packed.bwd), nat._ptr(self.packed.bias),
                               nat._ptr(self.bkgd), nat._ptr(self.ws), nat._ptr(self.rgb), nat._ptr(self.opacity),
                               nat._ptr(self.depth))
        nat._check(L.den_render_fwd(ctypes.byref(self.desc), ctypes.byref(self.io), st))
        args = (self.N, self.rd, ERR[self.fn[0]], ERR[self.fn[1]], int(self.has_bkgd), self.min_int, self.wl[0],
                self.wl[1], nat._ptr(self.rgb), nat._ptr(self.opacity), nat._ptr(self.channel),
                nat._ptr(self.target), nat._ptr(self.c), nat._ptr(self.ev_ws))
        nat._check(L.den_event_step_fwd(*args, nat._ptr(self.loss), st))
        nat._check(L.den_event_step_bwd(*args, nat._ptr(self.d_rgb), st))

    def backward(self):
        st = nat._stream(self.dev)
        gr = nat.RenderGrad(nat._ptr(self.d_rgb), None, None, nat._ptr(self.grad),
                            nat._ptr(self.grad_bkgd) if self.has_bkgd else None)
        nat._check(nat.lib().den_render_bwd(ctypes.byref(self.desc), ctypes.byref(self.io), ctypes.byref(gr), st))

    def allreduce(self):
        allreduce_mean(self.gbuf)

    def optimizer_step(self):
        self.t += 1
        nat.adam_step(self.flat, self.grad, self.m, self.v, self.lr, 0.9, 0.999, 1e-8, self.wd, self.t)
        if self.has_bkgd:
            g_orig = self.grad_bkgd * torch.sigmoid(self.bkgd_orig)  # softplus(beta=1) parametrisation chain rule
            nat.adam_step(self.bkgd_orig, g_orig.contiguous(), self.bm, self.bv, self.lr, 0.9, 0.999, 1e-8, 0.0,
                          self.t)
        self.packed.pack(self.flat)

    def step(self):
        self.forward()
        self.backward()
        self.allreduce()
        self.optimizer_step()
        return self.loss


def synthetic_batch(n_events, seed=1234, radius=4.03, device="cpu", rank=0, world=1):
    """Synthetic chair-like event batch.  Each event is one
    pixel seen from a camera on a sphere around the AABB; its four render
    timestamps (diff start/end, tv start/end) move the camera slightly.
    Returns the (4N,3) rays, jitter and the event fields; rank r of `world`
    gets the r-th contiguous shard of the events."""
    g = torch.Generator().manual_seed(seed)
    N = n_events * world
    v = torch.randn(N, 3, generator=g)
    c0 = v / v.norm(dim=-1, keepdim=True) * radius
    look = -c0 / c0.norm(dim=-1, keepdim=True) + (torch.rand(N, 3, generator=g) * 2 - 1) * math.sin(0.3)
    look = look / look.norm(dim=-1, keepdim=True)
    motion = torch.randn(4, N, 3, generator=g) * 0.01  # camera motion across the 4 timestamps
    o = (c0[None] + motion).reshape(4 * N, 3)
    d = look[None].expand(4, N, 3).reshape(4 * N, 3)
    jitter = torch.rand(4 * N, generator=g)
    pos = torch.rand(N, generator=g) < 0.5
    lid = torch.where(pos, 0.25, -0.25).float()
    end_ts = (torch.rand(N, generator=g, dtype=torch.float64) * 9e8 + 1e8).floor().long()
    start_ts = end_ts.double() - (-torch.log(torch.rand(N, generator=g, dtype=torch.float64)) * 1e6 + 1e3)
    ts_diff = end_ts.double() - start_ts
    sl = slice(rank * n_events, (rank + 1) * n_events)
    o4, d4, j4 = (t.reshape(4, N, *t.shape[1:])[:, sl].reshape(4 * n_events, *t.shape[1:]) for t in (o, d, jitter))
    return dict(rays_o=o4.to(device), rays_d=d4.to(device), jitter=j4.to(device), lid=lid[sl].to(device),
                end_ts=end_ts[sl].to(device), start_ts=start_ts[sl].to(device), ts_diff=ts_diff[sl].to(device))


def _look_at(centre, target_dir):
    """Camera-to-world rotation whose z axis (principal axis) is target_dir
    (x right, y down, as the reference's OpenCV-style intrinsics assume)."""
    z = target_dir / target_dir.norm(dim=-1, keepdim=True)
    up = torch.tensor([0.0, 0.0, 1.0]).expand_as(z)
    x = torch.linalg.cross(z, up)
    x = x / x.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    y = torch.linalg.cross(z, x)
    return torch.stack([x, y, z], dim=-1)  # columns = camera axes in world coordinates


def synthetic_events(n_events, seed=1234, radius=4.03, rank=0, world=1, img=800, focal=1111.0):
    """Synthetic chair-like RAW event batch, the form
    training_step receives: queued events (num_pos + num_neg = 1, polarity
    Bernoulli(0.5)), end_ts ~ U[1e8, 1e9] ns, intervals ~ Exp(1 ms) + 1 us (i64),
    the datamodule's normalized samples (ts_diff ~ Dirac(1), diff start ~ U,
    ts_subdiff ~ Tri(0, 1, mode 0), subdiff start ~ U; datamodule.py:151-197),
    pixel positions in an 800x800 image (f = 1111), and camera poses at the 4
    render timestamps: centres on a sphere around the AABB looking at the origin
    (+-0.3 rad), moving slightly between timestamps.  Rank r of `world` gets the
    r-th contiguous shard of the events (all 4 renders of an event on one rank)."""
    g = torch.Generator().manual_seed(seed)
    N = n_events * world
    v = torch.randn(N, 3, generator=g)
    c0 = v / v.norm(dim=-1, keepdim=True) * radius
    look = -c0 / c0.norm(dim=-1, keepdim=True) + (torch.rand(N, 3, generator=g) * 2 - 1) * math.sin(0.3)
    rot = _look_at(c0, look)
    motion = torch.randn(4, N, 3, generator=g) * 0.01
    pos = c0[None] + motion
    rot4 = rot[None].expand(4, N, 3, 3).contiguous()
    pixel = torch.rand(N, 2, generator=g) * img
    K = torch.tensor([[focal, 0.0, img / 2], [0.0, focal, img / 2], [0.0, 0.0, 1.0]])
    jitter = torch.rand(4, N, generator=g)
    num_pos = (torch.rand(N, generator=g) < 0.5).long()
    end_ts = (torch.rand(N, generator=g, dtype=torch.float64) * 9e8 + 1e8).long()
    start_ts = end_ts - (-torch.log(torch.rand(N, generator=g, dtype=torch.float64)) * 1e6 + 1e3).long()
    u = torch.rand(3, N, generator=g, dtype=torch.float64)
    norm = torch.stack([torch.ones(N, dtype=torch.float64), u[0], 1 - torch.sqrt(1 - u[1]), u[2]])
    sl = slice(rank * n_events, (rank + 1) * n_events)
    return dict(num_pos=num_pos[sl], num_neg=1 - num_pos[sl], end_ts=end_ts[sl], start_ts=start_ts[sl],
                normalized=norm[:, sl].contiguous(), position=pixel[sl], T_wc_position=pos[:, sl].contiguous(),
                T_wc_orientation=rot4[:, sl].contiguous(), intrinsics_inverse=torch.linalg.inv(K).contiguous(),
                jitter=jitter[:, sl].reshape(-1).contiguous())


# EDS-assumed DVS constants (reference scripts/eds_to_esim.py:68-79), the synthetic sensor
EDS_CALIBRATION = dict(
    input_time_const_eff_it_prod=(35e-12 * 25e-3) / 2000e-12,
    miller_time_const_eff_it_prod=(0.6e-12 * 25e-3) / 2000e-12,
    amplifier_gain=140.0, closed_loop_gain=1 / 0.7, output_time_const=25e-6,
    sf_cutoff_freq=16400.0, diff_amp_cutoff_freq=82000.0)


class _TargetCumprob(dict):
    __getattr__ = dict.__getitem__


class PixbwTrainStep:
    """Training step with the pixel-bandwidth model ON (BASELINE.json configs[2];
    DeblurENeRF.training_step, deblur_e_nerf.py:414-586, with
    render_log_intensity's pixel-bandwidth branch :1137-1151): per event, each of
    the 4 supervision timestamps [diff start (reset_diff), diff end, tv start,
    tv end] becomes S = it_sample_size intensity samples at the sample timestamps
    of PixelBandwidth.sample_intensity, i.e. S x N rays per render call and
    4 S N per step; the pixel-bandwidth filter turns them into log-intensities
    (den_pixbw_*), then the Huber diff + L1 TV losses, backward, all-reduce, Adam.

    Device ops: den_event_prep, den_pixbw_sample_ts, den_trajectory (the camera pose at every
    sample timestamp: LinearTrajectory.forward, trajectories.py:30-90), den_pixel_rays,
    den_render_fwd/bwd, den_pixbw_fwd/bwd, den_event_loss_fwd/bwd, den_adam_step,
    den_pack_weights, chained by torch.autograd -- the reference step's front end
    (render_train_pixels: trajectory -> pixel_params_to_ray -> render).
    """

    def __init__(self, n_events, it_sample_size=16, n_samples=128, radiance_dim=1, mode="bf16", seed=0,
                 device="cuda", aabb=(-1.5, -1.5, -1.5, 1.5, 1.5, 1.5), near=1.43, far=6.63, lr=0.01,
                 weight_decay=1e-6, loss_weight=(1.0, 1e-3), error_fn=("huber", "l1"), min_modeled_intensity=1e-3,
                 mean_contrast_threshold=0.25, min_ts=5e7, calibration=None):
        from .models.pixel_bandwidth import PixelBandwidth
        self.N, self.S, self.n_samples, self.rd = n_events, it_sample_size, n_samples, radiance_dim
        self.mode = nat.mode_id(mode)
        self.dev = torch.device(device)
        self.R = 4 * it_sample_size * n_events
        torch.manual_seed(seed)
        field = mlp.VanillaNeRFRadianceField(
            list(aabb), radiance_dim=radiance_dim, hidden_activation=torch.nn.Softplus(beta=100),
            density_activation=ngp.shifted_trunc_exp, radiance_activation=torch.nn.Softplus(beta=1), mode=mode)
        self.P = nat.param_count(radiance_dim)
        self.flat = field.flat_params.detach().to(self.dev).contiguous().requires_grad_(True)
        self.bkgd_orig = torch.full((radiance_dim,), math.log(math.expm1(1.0)), device=self.dev)
        self.gbuf = torch.zeros(self.P + radiance_dim, device=self.dev)
        self.m, self.v = torch.zeros_like(self.gbuf), torch.zeros_like(self.gbuf)
        self.t, self.lr, self.wd = 0, lr, weight_decay
        self.wl, self.fn, self.min_int = loss_weight, error_fn, min_modeled_intensity
        self.c = torch.tensor([mean_contrast_threshold], device=self.dev)
        self.ct = torch.tensor([mean_contrast_threshold] * 2, device=self.dev)
        self.tau = torch.zeros(1, dtype=torch.float64, device=self.dev)
        self.cfg = dict(mode=self.mode, rd=radiance_dim, aabb=list(aabb), near=near, far=far)
        self.packed = nat.PackedWeights(self.mode, radiance_dim, self.dev)
        self.packed.pack(self.flat.detach())
        cal = {k: np.array(v, dtype=np.float32) for k, v in (calibration or EDS_CALIBRATION).items()}
        self.pb = PixelBandwidth(None, torch.tensor(min_ts), 21.0, _TargetCumprob(max_sample_lifetime=0.95),
                                 calibration=cal).to(self.dev)
        for p in self.pb.parameters():
            p.requires_grad_(False)  # frozen in the synthetic configuration (synthetic.yaml:41-52)
        self.loss = torch.zeros(3, device=self.dev)

    def load_events(self, num_pos, num_neg, end_ts, start_ts, normalized, interval_gen, position, T_wc_position,
                    T_wc_orientation, T_wc_timestamp, intrinsics_inverse, jitter, channel=None):
        """Raw events (see synthetic_pixbw_events): interval_gen (S-1, N) f64 is the
        datamodule's normalized interval-generator sample (datamodule.py:199-211); the camera
        trajectory is the pose samples T_wc_position (C, 3), T_wc_orientation (C, 4) XYZW,
        T_wc_timestamp (C) ns (camera_poses.npz), looked up per sample timestamp by the
        LinearTrajectory mirror (den_trajectory); jitter (4, S N)."""
        from .data.datasets import CameraPose
        from .models.trajectories import LinearTrajectory
        d = self.dev
        i64 = lambda t: t.to(d, torch.int64).contiguous()
        f32 = lambda t: t.to(d, torch.float32).contiguous()
        self.ev = dict(num_pos=i64(num_pos), num_neg=i64(num_neg), end_ts=i64(end_ts), start_ts=i64(start_ts))
        self.norm = normalized.to(d, torch.float64).contiguous()
        self.gen = interval_gen.to(d, torch.float64).contiguous()
        self.position = f32(position)
        self.traj = LinearTrajectory(CameraPose.from_arrays(f32(T_wc_position), f32(T_wc_orientation),
                                                            i64(T_wc_timestamp))).to(d)
        self.K_inv = f32(intrinsics_inverse)
        self.jitter = f32(jitter).reshape(4, self.S * self.N)
        self.channel = None if channel is None else i64(channel)

    def _intensity_fn(self, g, bkgd):
        S, N = self.S, self.N

        def fn(ts):  # (S, N) f64 clamped sample timestamps -> intensity (S, N) (render_train_pixels)
            with torch.no_grad():  # (the pose path carries no gradient here: tau_r is frozen)
                pos, rot = self.traj(ts)
                o, dr = nat.pixel_rays(self.K_inv, self.position, pos.contiguous(), rot.contiguous())
            rgb, op, _ = nat.render(o.reshape(-1, 3), dr.reshape(-1, 3), self.jitter[g], bkgd, self.flat,
                                    self.cfg, self.packed, self.n_samples)
            if self.rd > 1:  # bayering (deblur_e_nerf.py:1223-1235)
                rad = rgb.view(S, N, self.rd).gather(2, self.channel.view(1, N, 1).expand(S, N, 1))[..., 0]
            else:
                rad = rgb.view(S, N)
            return (rad + self.min_int,)
        return fn

    def forward(self):
        e = self.ev
        prep = nat.event_prep(e["num_pos"], e["num_neg"], e["end_ts"], e["start_ts"], self.norm, self.ct, self.tau,
                              norm_c=self.c)
        # the gradient buffer holds d/d bkgd (post-softplus), as TrainStep's does
        bkgd = torch.nn.functional.softplus(self.bkgd_orig.detach()).requires_grad_(True)
        self.bkgd = bkgd
        y = [self.pb(self.gen, prep["render_ts"][g], self._intensity_fn(g, bkgd), reset_diff=(g == 0))[0]
             for g in range(4)]
        Ld = nat.EventLossFunction.apply(y[1] - y[0], prep["target"], self.c, None, self.fn[0])
        Lt = nat.EventLossFunction.apply(y[3] - y[2], None, self.c, None, self.fn[1])
        self.total = self.wl[0] * Ld + self.wl[1] * Lt
        self.loss = torch.stack([Ld.detach(), Lt.detach(), self.total.detach()])

    def backward(self):
        self.flat.grad = None
        self.total.backward()
        self.gbuf[: self.P].copy_(self.flat.grad)
        self.gbuf[self.P:].copy_(self.bkgd.grad)
        # drop the step's graph (and the render workspaces it holds) before the next forward
        self.total = None
        self.pb.reset_delta_log_it = self.pb.reset_delta_log_it.detach()

    def step(self):
        self.forward()
        self.backward()
        allreduce_mean(self.gbuf)
        self.t += 1
        with torch.no_grad():
            nat.adam_step(self.flat, self.gbuf[: self.P], self.m[: self.P], self.v[: self.P], self.lr, 0.9, 0.999,
                          1e-8, self.wd, self.t)
            g = (self.gbuf[self.P:] * torch.sigmoid(self.bkgd_orig.detach())).contiguous()  # softplus chain rule
            b, bm, bv = self.bkgd_orig.detach(), self.m[self.P:], self.v[self.P:]
            nat.adam_step(b, g, bm, bv, self.lr, 0.9, 0.999, 1e-8, 0.0, self.t)
            self.packed.pack(self.flat.detach())
        return self.loss


def rotmat_to_quat_xyzw(R):
    """(..., 3, 3) rotation matrices -> (..., 4) unit quaternions in RoMa's XYZW order (Shepperd's
    method, the largest of the four candidate pivots); synthetic pose data only."""
    m = R
    tr = m[..., 0, 0] + m[..., 1, 1] + m[..., 2, 2]
    cands = torch.stack([tr, m[..., 0, 0], m[..., 1, 1], m[..., 2, 2]], dim=-1)
    k = cands.argmax(dim=-1)
    s0 = torch.sqrt((1 + tr).clamp_min(1e-12)) * 2
    s1 = torch.sqrt((1 + m[..., 0, 0] - m[..., 1, 1] - m[..., 2, 2]).clamp_min(1e-12)) * 2
    s2 = torch.sqrt((1 + m[..., 1, 1] - m[..., 0, 0] - m[..., 2, 2]).clamp_min(1e-12)) * 2
    s3 = torch.sqrt((1 + m[..., 2, 2] - m[..., 0, 0] - m[..., 1, 1]).clamp_min(1e-12)) * 2
    q0 = torch.stack([(m[..., 2, 1] - m[..., 1, 2]) / s0, (m[..., 0, 2] - m[..., 2, 0]) / s0,
                      (m[..., 1, 0] - m[..., 0, 1]) / s0, s0 / 4], -1)
    q1 = torch.stack([s1 / 4, (m[..., 0, 1] + m[..., 1, 0]) / s1, (m[..., 0, 2] + m[..., 2, 0]) / s1,
                      (m[..., 2, 1] - m[..., 1, 2]) / s1], -1)
    q2 = torch.stack([(m[..., 0, 1] + m[..., 1, 0]) / s2, s2 / 4, (m[..., 1, 2] + m[..., 2, 1]) / s2,
                      (m[..., 0, 2] - m[..., 2, 0]) / s2], -1)
    q3 = torch.stack([(m[..., 0, 2] + m[..., 2, 0]) / s3, (m[..., 1, 2] + m[..., 2, 1]) / s3, s3 / 4,
                      (m[..., 1, 0] - m[..., 0, 1]) / s3], -1)
    q = torch.where((k == 0)[..., None], q0, torch.where((k == 1)[..., None], q1, torch.where((k == 2)[..., None], q2, q3)))
    return q / q.norm(dim=-1, keepdim=True)


def synthetic_trajectory(speed=5.0, radius=4.03, n_poses=401, t_end=1.2e9, seed=7):
    """A camera_poses.npz-shaped trajectory: the camera orbits the AABB centre at `radius` with
    `speed` units/s and a slow elevation swing, looking at the origin (x right, y down); pose
    samples every t_end / (n_poses - 1) ns -> T_wc_position (C, 3) f32, T_wc_orientation (C, 4)
    XYZW f32, T_wc_timestamp (C) i64."""
    g = torch.Generator().manual_seed(seed)
    phase = float(torch.rand(1, generator=g)) * 2 * math.pi
    t = torch.linspace(0.0, t_end, n_poses, dtype=torch.float64)
    theta = phase + speed / radius * t * 1e-9
    elev = 0.35 + 0.25 * torch.sin(0.37 * t * 1e-9 + phase)
    c = torch.stack([torch.cos(theta) * torch.cos(elev), torch.sin(theta) * torch.cos(elev), torch.sin(elev)], -1)
    c = (c * radius).float()
    rot = _look_at(c, -c)
    return dict(T_wc_position=c.contiguous(), T_wc_orientation=rotmat_to_quat_xyzw(rot).float().contiguous(),
                T_wc_timestamp=t.round().long())


def synthetic_pixbw_events(n_events, it_sample_size=16, seed=1234, rank=0, world=1, speed=5.0):
    """synthetic_events plus the pixel-bandwidth inputs: the (S-1, N) interval generator sample
    (Triangular(0,1) about 0.5, datamodule.py:199-211) and ONE camera trajectory for all events
    (synthetic_trajectory: camera_poses.npz's arrays; the pose of each sample timestamp comes from
    it, as render_train_pixels looks it up); jitter covers the 4 x S x N rays.  Every rank holds the
    same trajectory and its shard of the events."""
    S = it_sample_size
    b = synthetic_events(n_events, seed=seed, rank=rank, world=world)
    g = torch.Generator().manual_seed(seed + 1)
    Nt = n_events * world
    u = torch.rand(S - 1, Nt, generator=g, dtype=torch.float64)
    gen = torch.where(u < 0.5, torch.sqrt(u / 2), 1 - torch.sqrt((1 - u) / 2))
    jit = torch.rand(4, S, Nt, generator=g)
    sl = slice(rank * n_events, (rank + 1) * n_events)
    for k in ("jitter", "T_wc_position", "T_wc_orientation"):
        b.pop(k)
    b.update(interval_gen=gen[:, sl].contiguous(), jitter=jit[:, :, sl].reshape(4, -1).contiguous(),
             **synthetic_trajectory(speed=speed, seed=seed + 2))
    return b
