"""Event-generation model parameters (reference models/event_generation_params.py).

``ContrastThreshold`` and ``RefractoryPeriod`` keep the reference's constructor
arguments, parametrisations (softplus / scaled-shifted sigmoid on the scalar
parameters, utils/modules.py) and properties.  Their per-event arithmetic runs in
libden.so: ``prepare_events`` is the fused device step of
DeblurENeRF.training_step lines 414-455 (contrast threshold, refractory delay,
diff / subdiff timestamps and the normalised diff target, ``den_event_prep``);
each module's ``forward`` is the same kernel with only its own outputs kept.
The transforms of the <= 3 scalar parameters stay in PyTorch (as for the render
background).  Forward only: the configurations in BASELINE.json freeze these
parameters for the synthetic path (configs/train/synthetic.yaml:29-40).
"""
import os
import warnings

import numpy as np
import torch

from .. import _native
from ..utils import modules


def _load_calibration(dataset_directory, calibration):
    if calibration is not None:
        return calibration
    # data/datasets.py:105-111 (np.load of a plain .npz; no pickles)
    return dict(np.load(os.path.join(dataset_directory, "camera_calibration.npz")))


class ContrastThreshold(torch.nn.Module):
    """event_generation_params.py:8-118."""

    def __init__(self, dataset_directory=None, parameterize_mean_ct=True, calibration=None):
        super().__init__()
        cal = _load_calibration(dataset_directory, calibration)
        pos = torch.as_tensor(np.asarray(cal["pos_contrast_threshold"]))
        neg = torch.as_tensor(np.asarray(cal["neg_contrast_threshold"]))
        ratio, mean = pos / neg, (pos + neg) / 2
        assert ratio > 0 and mean > 0
        self.register_buffer("init_p2n_contrast_threshold_ratio", ratio, persistent=False)
        self.register_buffer("init_mean_contrast_threshold", mean, persistent=False)
        softplus = modules.Softplus(beta=1)
        self.p2n_contrast_threshold_ratio = torch.nn.Parameter(ratio.clone())
        torch.nn.utils.parametrize.register_parametrization(self, "p2n_contrast_threshold_ratio", softplus)
        self.parameterize_mean_ct = parameterize_mean_ct
        if parameterize_mean_ct:
            self.mean_contrast_threshold = torch.nn.Parameter(mean.clone())
            torch.nn.utils.parametrize.register_parametrization(self, "mean_contrast_threshold", softplus)
        else:
            self.register_buffer("_neg_contrast_threshold", neg, persistent=False)

    @property
    def neg_contrast_threshold(self):
        if self.parameterize_mean_ct:
            return 2 * self.mean_contrast_threshold / (self.p2n_contrast_threshold_ratio + 1)
        return self._neg_contrast_threshold

    @property
    def pos_contrast_threshold(self):
        return self.p2n_contrast_threshold_ratio * self.neg_contrast_threshold

    @property
    def mean_ct(self):
        if self.parameterize_mean_ct:
            return self.mean_contrast_threshold
        return (self.pos_contrast_threshold + self.neg_contrast_threshold) / 2

    @property
    def ref_p2n_contrast_threshold_ratio(self):
        return self.p2n_contrast_threshold_ratio / self.init_p2n_contrast_threshold_ratio

    @property
    def delta_mean_contrast_threshold(self):
        return self.mean_ct - self.init_mean_contrast_threshold

    def device_params(self, device):
        """(2) f32 [C+, C-] on the device, as den_event_prep reads them."""
        with torch.no_grad():
            return torch.stack([self.pos_contrast_threshold, self.neg_contrast_threshold]).float().to(device)

    def forward(self, input_event):
        ev = dict(input_event)
        out = _prep_only(ev, self.device_params(ev["end_ts"].device), None)
        ev["log_intensity_diff"] = out["lid"]
        ev.pop("num_pos")
        ev.pop("num_neg")
        return ev


class RefractoryPeriod(torch.nn.Module):
    """event_generation_params.py:121-237.  ``max_refractory_period`` is the cached
    ``max_refractory_period.pt``, else extracted from ``raw_events.npz`` on the GPU
    (datasets.Event.extract_max_refractory_period, den_max_refractory_period) and cached, as the
    reference does (:135-149); it may also be given directly."""
    REFRACTORY_PERIOD_KEY = "refractory_period"
    REDEFINED_CALIBRATED_REFRACTORY_PERIOD_FACTOR = 0.999
    MIN_SCALED_SHIFTED_SIGMOID_GRAD_MAGNITUDE = 0.0001

    def __init__(self, dataset_directory=None, max_refractory_period=None, calibration=None):
        super().__init__()
        cal = _load_calibration(dataset_directory, calibration)
        tau = torch.as_tensor(np.asarray(cal[self.REFRACTORY_PERIOD_KEY]))
        if max_refractory_period is None:
            from ..data import datasets
            max_refractory_period = datasets.Event.load_max_refractory_period(dataset_directory)
            if max_refractory_period is None:
                raw_events = datasets.Event.load_raw_events(dataset_directory)
                max_refractory_period = datasets.Event.extract_max_refractory_period(raw_events, cal)
                datasets.Event.save_max_refractory_period(max_refractory_period, dataset_directory)
        mx = torch.as_tensor(max_refractory_period)
        if not (0 <= tau < mx):
            warnings.warn(f"Calibrated refractory period ({tau}) >= Max. possible refractory period ({mx}).")
            tau = self.REDEFINED_CALIBRATED_REFRACTORY_PERIOD_FACTOR * mx
            warnings.warn(f"Redefining calibrated refractory period to {self.REDEFINED_CALIBRATED_REFRACTORY_PERIOD_FACTOR}"
                          f" of max. possible refractory period ({tau}).")
        self.register_buffer("init_refractory_period", tau, persistent=False)
        self.register_buffer("max_refractory_period", mx, persistent=False)
        self.register_buffer("max_scaled_logit_magnitude",
                             torch.tensor(self.MIN_SCALED_SHIFTED_SIGMOID_GRAD_MAGNITUDE).logit().abs(),
                             persistent=False)
        self._refractory_period = torch.nn.Parameter(tau.to(torch.float64))
        torch.nn.utils.parametrize.register_parametrization(
            self, "_refractory_period", modules.ScaledShiftedSigmoid(low=0, high=mx))
        self.clamp_refractory_period()

    @torch.no_grad()
    def clamp_refractory_period(self):
        orig = self.parametrizations._refractory_period.original
        scaled = orig / self.max_refractory_period
        m = self.max_scaled_logit_magnitude
        orig.copy_(self.max_refractory_period * scaled.clamp(min=-m, max=m))

    @property
    def refractory_period(self):
        self.clamp_refractory_period()
        return self._refractory_period

    @property
    def delta_refractory_period(self):
        return self.refractory_period - self.init_refractory_period

    def device_params(self, device):
        """(1) f64 tau_r (ns) on the device."""
        with torch.no_grad():
            return self.refractory_period.detach().to(torch.float64).reshape(1).to(device)

    def forward(self, input_event):
        ev = dict(input_event)
        dev = ev["end_ts"].device
        n = ev["end_ts"].numel()
        zeros = torch.zeros(n, dtype=torch.int64, device=dev)
        e2 = dict(ev, num_pos=zeros, num_neg=zeros)
        out = _prep_only(e2, torch.zeros(2, device=dev), self.device_params(dev))
        ev["start_ts"] = out["start_ts"]
        return ev


def _prep_only(ev, ct, refractory):
    dev = ev["end_ts"].device
    n = ev["end_ts"].numel()
    if refractory is None:
        refractory = torch.zeros(1, dtype=torch.float64, device=dev)
    start = ev["start_ts"]
    if start.dtype != torch.int64:
        raise _native.DenError("start_ts must be the raw i64 event timestamps")
    return _native.event_prep(ev["num_pos"].contiguous(), ev["num_neg"].contiguous(), ev["end_ts"].contiguous(),
                              start.contiguous(), torch.zeros(4, n, dtype=torch.float64, device=dev), ct, refractory,
                              has_diff=False, has_tv=False)


def prepare_events(contrast_threshold, refractory_period, event, normalized, loss_weight=(1.0, 1e-3),
                   normalize_target=True):
    """Fused deblur_e_nerf.py:414-455 (+ loss.py:74-77's target): raw events
    (num_pos, num_neg, end_ts, start_ts i64) and the normalized (4,N) f64 samples
    -> dict(lid, start_ts, render_ts (4,N), ts_diff, ts_subdiff, target)."""
    dev = event["end_ts"].device
    ct = contrast_threshold.device_params(dev)
    c = contrast_threshold.mean_ct.detach().float().reshape(1).to(dev) if normalize_target else \
        torch.ones(1, device=dev)
    return _native.event_prep(event["num_pos"], event["num_neg"], event["end_ts"], event["start_ts"], normalized, ct,
                              refractory_period.device_params(dev), norm_c=c if loss_weight[0] > 0 else None,
                              has_diff=loss_weight[0] > 0, has_tv=loss_weight[1] > 0)
