"""The evaluation's affine log-intensity alignment (models/deblur_e_nerf.affine_log_intensity_correction,
the reference's deblur_e_nerf.py:705-833 without the black-level LM refinement): host-side f64
least squares, checked on CPU against a known affine map and against the closed-form regression."""
import math

import torch

from deblur_e_nerf.models.deblur_e_nerf import affine_log_intensity_correction


def test_recovers_known_affine_map_grayscale():
    g = torch.Generator().manual_seed(3)
    target = torch.rand(3, 20, 24, generator=g, dtype=torch.float64) * 0.9 + 0.05
    # pred = exp((log target - b) / a): the correction must find gamma = a, scale = e^b
    a, b = 0.7, -0.4
    pred = ((target.log() - b) / a).exp()
    corr, gamma, scale = affine_log_intensity_correction(pred, target)
    assert corr.shape == (3, 1, 20, 24)
    assert abs(float(gamma[0]) - a) < 1e-9 and abs(float(scale[0]) - math.exp(b)) < 1e-9
    assert float((corr[:, 0] - target.double()).abs().max()) < 1e-9


def test_matches_closed_form_regression_with_gain_exposure():
    g = torch.Generator().manual_seed(4)
    target = torch.rand(2, 16, 16, generator=g) * 0.8 + 0.1
    pred = (target + torch.rand(2, 16, 16, generator=g) * 0.05).clamp(0.01, 1)
    gep = torch.tensor([1.0, 2.0])
    corr, gamma, scale = affine_log_intensity_correction(pred, target, gain_exposure_prod=gep)
    lg = (gep / gep.mean()).log().view(2, 1, 1).double()
    x, y = pred.double().log().reshape(-1), (target.double().log() - lg).reshape(-1)
    xm, ym = x.mean(), y.mean()
    a = ((x - xm) * (y - ym)).sum() / ((x - xm) ** 2).sum()
    b = ym - a * xm
    assert abs(float(gamma[0] - a)) < 1e-6 and abs(float(scale[0].log() - b)) < 1e-6
    want = ((a * pred.double().log() + b) + lg).exp()
    assert float((corr[:, 0] - want).abs().max()) < 1e-6


def test_bayer_shared_scale_per_channel_offsets():
    g = torch.Generator().manual_seed(5)
    target = torch.rand(1, 3, 10, 12, generator=g, dtype=torch.float64) * 0.9 + 0.05
    offs = torch.tensor([0.1, -0.2, 0.3], dtype=torch.float64).view(1, 3, 1, 1)
    pred = ((target.log() - offs) / 1.25).exp()
    corr, gamma, scale = affine_log_intensity_correction(pred, target, has_bayer_filter=True)
    assert gamma.shape == (1,) and scale.shape == (3,)
    assert abs(float(gamma[0]) - 1.25) < 1e-9
    assert torch.allclose(scale.log(), offs.view(3).double(), atol=1e-9)
    # per-channel scale requested: one (gamma, scale) pair per channel
    _, gamma3, scale3 = affine_log_intensity_correction(pred, target, has_bayer_filter=True,
                                                        per_channel_log_it_scale=True)
    assert gamma3.shape == (3,) and scale3.shape == (3,)
