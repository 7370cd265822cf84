"""The evaluation path: DeblurENeRF.render_image_eval against the reference's evaluation_step render
(tests/golden/eval_rd*.npz, make_golden.gen_eval: render_pixels of the meshgrid pixel positions at
one camera pose, eval mode, after one occupancy-grid update) and Metric.compute (den_image_error)
against the reference's formulas (loss_metric/metric.py:68-72: torch l1_loss; torchmetrics psnr
with data_range = max - min, per image over (C, H, W), mean over the batch).  Needs an MI355X."""
import math
import os

import numpy as np
import pytest
import torch

from test_deblur_gpu import build_model
from test_nerfacc_gpu import _Draws

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("rd", [1, 3])
def test_render_image_eval_matches_reference(golden_dir, rd, monkeypatch):
    """F32 at the north-star 1e-4 relative (image-wise)."""
    from deblur_e_nerf.external import marching
    z = np.load(os.path.join(golden_dir, f"eval_rd{rd}.npz"))
    m = build_model(z)
    monkeypatch.setattr(marching, "_uniform", _Draws([z["occ_u"]]))
    m.nerf.update_occ_grid(step=0, T_wc_position=m.trajectory.T_wc_position)
    H, W = int(z["H"]), int(z["W"])
    with torch.no_grad():
        img = m.render_image_eval(torch.from_numpy(z["kinv"]), torch.from_numpy(z["pos"]), torch.from_numpy(z["rot"]),
                                  H, W)
    torch.cuda.synchronize()
    ref = torch.from_numpy(z["img"]).double()
    got = img.detach().cpu().double()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    e = float((got - ref).norm() / ref.norm())
    emax = float((got - ref).abs().max())
    print(f"[eval rd={rd}] {tuple(got.shape)} image rel err {e:.2e}, max abs {emax:.2e}, "
          f"opacity range {z['opacity'].min():.3f}..{z['opacity'].max():.3f}")
    assert e <= 1e-4


def _ref_metric(pred, target, lo, hi):
    """metric.py:68-72 in f64: l1_loss over everything; psnr per image (dims 1..3), then the mean."""
    p, t = pred.double(), target.double()
    while t.dim() < 4:
        p, t = p[None], t[None]
    l1 = float((p - t).abs().mean())
    mse = ((p - t) ** 2).flatten(1).mean(1)
    psnr = float((10 * torch.log10((hi - lo) ** 2 / mse)).mean())
    return l1, psnr


@pytest.mark.parametrize("shape", [(40, 56), (1, 40, 56), (3, 33, 17), (4, 3, 64, 48), (2, 1, 128, 96)])
def test_metric_matches_reference_formula(shape):
    from deblur_e_nerf.loss_metric.metric import Metric, psnr
    g = torch.Generator().manual_seed(sum(shape))
    target = torch.rand(*shape, generator=g) * 0.8 + 0.1
    pred = (target + torch.randn(*shape, generator=g) * 0.05).clamp(0, 1)
    lo, hi = 0.05, 0.95
    got = Metric().compute(pred.to(DEV), target.to(DEV), lo, hi)
    l1, ps = _ref_metric(pred, target, lo, hi)
    print(f"[{shape}] l1 {float(got.l1):.6e} vs {l1:.6e}; psnr {float(got.psnr):.6f} vs {ps:.6f} dB")
    assert abs(float(got.l1) - l1) <= 1e-6 * l1
    assert abs(float(got.psnr) - ps) <= 1e-6 * abs(ps)
    if len(shape) < 4 or shape[0] == 1:
        assert abs(psnr(pred.to(DEV), target.to(DEV), 1.0) - _ref_metric(pred, target, 0.0, 1.0)[1]) <= 1e-5


def test_metric_identical_images_and_degenerate_range():
    """Equal images: the reference's PSNR is +inf (torchmetrics divides by a zero MSE); an empty data
    range is refused by its assertion, as here."""
    from deblur_e_nerf.loss_metric.metric import Metric
    x = torch.rand(1, 3, 16, 16, device=DEV)
    assert math.isinf(float(Metric().compute(x, x.clone(), 0.0, 1.0).psnr))
    with pytest.raises(AssertionError):
        Metric().compute(x, x, 1.0, 1.0)
