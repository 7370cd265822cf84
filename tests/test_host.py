"""Host-side logic that needs no GPU: the module mirrors' parametrisations and
properties against the reference semantics, synthetic-input invariants, and
the device ops' refusal of host tensors (there is no CPU fallback)."""
import numpy as np
import pytest
import torch


def _cal():
    return dict(pos_contrast_threshold=np.float32(0.25), neg_contrast_threshold=np.float32(0.2),
                refractory_period=np.int64(250000))


def test_contrast_threshold_mirror_properties():
    """event_generation_params.py:86-104: C- = 2 Cbar / (r + 1), C+ = r C-, and the
    calibrated values round-trip through the softplus parametrisation."""
    from deblur_e_nerf.models.event_generation_params import ContrastThreshold
    ct = ContrastThreshold(calibration=_cal(), parameterize_mean_ct=True)
    assert torch.allclose(ct.pos_contrast_threshold, torch.tensor(0.25), rtol=1e-6)
    assert torch.allclose(ct.neg_contrast_threshold, torch.tensor(0.2), rtol=1e-6)
    assert torch.allclose(ct.mean_ct, torch.tensor(0.225), rtol=1e-6)
    assert torch.allclose(ct.ref_p2n_contrast_threshold_ratio, torch.tensor(1.0), rtol=1e-6)
    legacy = ContrastThreshold(calibration=_cal(), parameterize_mean_ct=False)
    assert torch.allclose(legacy.mean_ct, torch.tensor(0.225), rtol=1e-6)


def test_refractory_period_mirror_clamps_and_redefines():
    """event_generation_params.py:150-163, 204-224: an out-of-range calibration is
    redefined to 0.999 x max; the scaled logit is clamped so the sigmoid gradient
    stays >= 1e-4."""
    from deblur_e_nerf.models.event_generation_params import RefractoryPeriod
    rp = RefractoryPeriod(calibration=_cal(), max_refractory_period=torch.tensor(1000000))
    assert abs(float(rp.refractory_period) - 250000.0) < 1e-3
    bad = dict(_cal(), refractory_period=np.int64(2000000))
    rp2 = RefractoryPeriod(calibration=bad, max_refractory_period=torch.tensor(1000000))
    assert abs(float(rp2.refractory_period) - 0.999e6) < 1.0
    with torch.no_grad():
        rp.parametrizations._refractory_period.original.fill_(1e12)
    tau = float(rp.refractory_period)
    s = tau / 1e6
    assert s * (1 - s) >= 1e-4 * 0.999


def test_synthetic_events_are_well_formed():
    from deblur_e_nerf.train import synthetic_events, synthetic_pixbw_events
    b = synthetic_events(64)
    assert torch.all(b["num_pos"] + b["num_neg"] == 1)
    assert torch.all(b["end_ts"] > b["start_ts"])
    assert b["normalized"].shape == (4, 64) and torch.all(b["normalized"][0] == 1.0)
    assert torch.all((b["normalized"] >= 0) & (b["normalized"] <= 1))
    R = b["T_wc_orientation"]
    eye = torch.eye(3).expand_as(R)
    assert torch.allclose(R.transpose(-1, -2) @ R, eye, atol=1e-5)  # rotations
    p = synthetic_pixbw_events(32, 16)
    assert p["interval_gen"].shape == (15, 32) and p["jitter"].numel() == 4 * 16 * 32
    assert torch.all((p["interval_gen"] >= 0) & (p["interval_gen"] <= 1))


def test_device_ops_refuse_host_tensors():
    from deblur_e_nerf import _native as nat
    x = torch.zeros(8, dtype=torch.int64)
    with pytest.raises(nat.DenError):
        nat.event_prep(x, x, x, x, torch.zeros(4, 8, dtype=torch.float64), torch.zeros(2),
                       torch.zeros(1, dtype=torch.float64))
    with pytest.raises(nat.DenError):
        nat.pixel_rays(torch.eye(3), torch.zeros(5, 2), torch.zeros(5, 3), torch.zeros(5, 3, 3))
