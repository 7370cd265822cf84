"""Oracle: pixel-bandwidth sensor model (4th-order LTV low-pass, FOH-discretised)
-- CPU PyTorch restatement (test infrastructure, see oracle/__init__.py).

Reference semantics followed (deblur_e_nerf/..., file:line):
* sample lifetimes / timestamps      models/pixel_bandwidth.py:298-367
* linearised continuous system       models/pixel_bandwidth.py:181-228
* FOH discretisation (efficient)     utils/control.py:87-93, 109-114
* weights from discretised system    models/pixel_bandwidth.py:260-296
* normalised weighted log-sum, reset models/pixel_bandwidth.py:398-448
* forward glue                       models/pixel_bandwidth.py:450-494

Parameters are passed post-parametrisation (softplus already applied), as the
reference reads them through ``torch.nn.utils.parametrize``.
"""
import math

import numpy as np
import torch

NS_TO_S = 1e-9
PARAM_NAMES = ("tau_mil_it_eff_prod", "A_amp_inv", "A_loop_inv", "tau_out", "tau_sf", "tau_diff")


def calib_to_params(calib):
    """Camera-calibration constants -> the module's parameter values
    (pixel_bandwidth.py:113-117)."""
    k_in = float(calib["input_time_const_eff_it_prod"])
    return dict(
        tau_in_it_eff_prod=k_in,
        tau_mil_it_eff_prod=float(calib["miller_time_const_eff_it_prod"]),
        A_amp_inv=1.0 / float(calib["amplifier_gain"]),
        A_loop_inv=float(calib["closed_loop_gain"]) / float(calib["amplifier_gain"]),
        tau_out=float(calib["output_time_const"]),
        tau_sf=1.0 / (2 * math.pi * float(calib["sf_cutoff_freq"])),
        tau_diff=1.0 / (2 * math.pi * float(calib["diff_amp_cutoff_freq"])),
    )


def sample_timestamps(gen, output_ts, omega_c_min, max_cumprob=0.95):
    """gen (S-1, N) f64 in [0,1], output_ts (N) f64 ns -> sample_ts (S, N) f64 ns
    (un-clamped; the renderer sees ts.clamp(min=min_ts))."""
    S = gen.shape[0] + 1
    b = torch.linspace(1, 0, S, dtype=gen.dtype).view(-1, *([1] * (gen.dim() - 1)))
    v = torch.lerp(b[:-1], b[1:], gen)
    m = torch.lerp(v[:-1], v[1:], 0.5)
    n = torch.cat([torch.ones_like(m[:1]), m, torch.zeros_like(m[:1])], dim=0)
    # torch.distributions.Exponential stores a Python-float rate as a float32
    # tensor, and the cumulative-probability buffer is a float32 tensor
    # (pixel_bandwidth.py:81-83, 344-350): both enter as f32-rounded values.
    rate = float(np.float32(NS_TO_S * omega_c_min))
    p = float(np.float32(max_cumprob)) * n
    lifetime = -torch.log1p(-p) / rate
    return output_ts - lifetime


def _system(I_lin, prm, with_sf):
    """Continuous A (..., 4, 4), B (..., 4, 1), C (o, 4) linearised at I_lin."""
    tau_in = prm["tau_in_it_eff_prod"] / I_lin
    tau_mil = prm["tau_mil_it_eff_prod"] / I_lin
    P = (tau_in + tau_mil) * prm["tau_out"]
    A_amp = 1 / prm["A_amp_inv"]
    A_loop = 1 / prm["A_loop_inv"]
    two_zw = (tau_in + prm["tau_out"] + (A_amp + 1) * tau_mil) / P
    w2 = (A_loop + 1) / P
    w_sf = 1 / prm["tau_sf"]
    w_df = 1 / prm["tau_diff"]
    z = torch.zeros_like(I_lin)
    o = torch.ones_like(I_lin)
    wsf = w_sf * o
    wdf = w_df * o
    A = torch.stack([
        torch.stack([-two_zw, -w2, z, z], -1),
        torch.stack([o, z, z, z], -1),
        torch.stack([z, wsf, -wsf, z], -1),
        torch.stack([z, z, wdf, -wdf], -1)], -2)
    B = torch.stack([w2, z, z, z], -1)[..., None]
    C = torch.tensor([[0, 0, 1, 0], [0, 0, 0, 1]], dtype=I_lin.dtype)
    if not with_sf:
        C = C[1:]
    return A, B, C


def foh_discretise(A, B, dt):
    """Efficient FOH with state preservation: Ad = e^{A dt}, Bd = G1 - G2, Btd = G2
    with M = A^-1 B, G1 = (Ad - I) M, G2 = (A dt)^-1 G1 - M."""
    Adt = A * dt[..., None, None]
    Phi = torch.linalg.matrix_exp(Adt)
    M = torch.linalg.solve(A, B)
    G1 = (Phi - torch.eye(A.shape[-1], dtype=A.dtype)) @ M
    G2 = torch.linalg.solve(Adt, G1) - M
    return Phi, G1 - G2, G2


def weights(I, sample_ts, prm, with_sf, dt_dtype=None):
    """I (S, N), sample_ts (S, N) f64 ns -> unnormalised weights (S, N, o).
    dt_dtype: dtype the f64 timestamp differences are cast to (the reference casts
    them to the intensity dtype, pixel_bandwidth.py:486; f32 in its training runs)."""
    dt = NS_TO_S * torch.diff(sample_ts, dim=0).to(dt_dtype or I.dtype).to(I.dtype)
    A, B, C = _system(I[1:], prm, with_sf)
    Ad, Bd, Btd = foh_discretise(A, B, dt)
    S = I.shape[0]
    w = [None] * S
    w[S - 1] = (C @ Btd[S - 2])[..., 0]
    c = C.expand(*I.shape[1:], *C.shape)
    for i in range(S - 2, 0, -1):
        c_next = c @ Ad[i]
        w[i] = (c @ Bd[i] + c_next @ Btd[i - 1])[..., 0]
        c = c_next
    w[0] = (c @ Bd[0])[..., 0]
    return torch.stack(w, 0)


class PixelBandwidthOracle:
    """Stateful wrapper mirroring PixelBandwidth.forward's reset semantics."""

    def __init__(self, prm, min_ts, f_c_dominant_min=21.0, max_cumprob=0.95, dt_dtype=None):
        self.prm = prm
        self.dt_dtype = dt_dtype
        self.min_ts = min_ts
        self.omega_c_min = 2 * math.pi * f_c_dominant_min
        self.max_cumprob = max_cumprob
        self.reset_delta_log_it = None
        self.reset_ts = None

    def __call__(self, gen, output_ts, intensity_fn, reset_diff=False):
        with torch.no_grad():
            sts = sample_timestamps(gen, output_ts, self.omega_c_min, self.max_cumprob)
        I = intensity_fn(torch.clamp(sts, min=float(self.min_ts)))
        w = weights(I, sts, self.prm, with_sf=reset_diff, dt_dtype=self.dt_dtype)
        wn = w / w.sum(dim=0, keepdim=True)
        y = (wn * torch.log(I)[..., None]).sum(dim=0)
        if reset_diff:
            self.reset_delta_log_it = y[..., 1] - y[..., 0]
            self.reset_ts = output_ts
            return y[..., 0]
        dt = (output_ts - self.reset_ts).to(self.dt_dtype or y.dtype).to(y.dtype)
        assert torch.all(dt >= 0)
        return y[..., 0] - self.reset_delta_log_it * torch.exp(-(1 / self.prm["tau_diff"]) * (NS_TO_S * dt))
