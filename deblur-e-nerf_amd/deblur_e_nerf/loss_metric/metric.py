"""Evaluation metrics -- mirror of the reference's loss_metric/metric.py (Metric, :8-92).

Same ``compute(pred_img, target_img, min_target_val, max_target_val) -> EasyDict`` with the
reference's input checks and metrics:

* ``l1``: torch l1_loss (mean absolute error over everything);
* ``psnr``: torchmetrics 0.6.2 functional.psnr with ``data_range = max - min``, per image over
  (C, H, W), mean over the batch: 10 log10(range^2 / MSE) -- the per-image error sums run in
  den_image_error;
* ``ssim``: torchmetrics 0.6.2 functional.ssim with ``data_range = max_target_val`` (11 x 11
  Gaussian window, sigma 1.5, k1 0.01, k2 0.03; mean over the images of each one's mean index) --
  den_ssim.  torchmetrics is not installed here, so its formula is restated (parity unpinned; the
  restatement in oracle/metrics.py is the checker);
* ``lpips``: computed only when the ``lpips`` package (and the pretrained network weights it
  downloads) is available, as the reference does; this image has neither, so the metric is absent
  from the results rather than faked.
"""
import math

import torch

from .. import _native
from ..utils.easydict import EasyDict

try:
    import lpips as _lpips
except ImportError:  # pragma: no cover - not in this image
    _lpips = None


class Metric(torch.nn.Module):
    METRIC_NAMES = ["l1", "psnr", "ssim"] + (["lpips"] if _lpips is not None else [])

    def __init__(self, metric_lpips_net=None):
        super().__init__()
        self.lpips_net = metric_lpips_net
        self.lpips = None
        if _lpips is not None and metric_lpips_net is not None:
            self.lpips = _lpips.LPIPS(net=metric_lpips_net)
            for p in self.lpips.parameters():
                p.requires_grad_(False)

    def init_batch_metric(self):
        return EasyDict({name: [] for name in self.METRIC_NAMES})

    def compute(self, pred_img, target_img, min_target_val, max_target_val):
        assert pred_img.shape == target_img.shape
        assert 2 <= target_img.dim() <= 4
        if target_img.dim() > 2:
            assert target_img.shape[-3] in (1, 3)
        assert 0 <= min_target_val < max_target_val
        assert bool(torch.all(min_target_val <= target_img)) and bool(torch.all(target_img <= max_target_val))
        if target_img.dim() < 4:
            shape = (4 - target_img.dim()) * (1,) + tuple(target_img.shape)
            pred_img, target_img = pred_img.reshape(shape), target_img.reshape(shape)
        B = target_img.shape[0]
        pix = target_img[0].numel()
        err = _native.image_error(pred_img, target_img).cpu()
        rng = float(max_target_val - min_target_val)
        # a zero MSE gives +inf, as torchmetrics' psnr does (a division by zero in torch)
        psnr = [10.0 * math.log10(rng * rng / (float(err[b, 0]) / pix)) if float(err[b, 0]) > 0 else math.inf
                for b in range(B)]
        metric = EasyDict({})
        metric.l1 = torch.tensor(float(err[:, 1].sum()) / (B * pix))
        metric.psnr = torch.tensor(sum(psnr) / B)
        H, W = target_img.shape[-2:]
        if min(H, W) >= _native.SSIM_WIN:
            metric.ssim = torch.tensor(float(_native.ssim(pred_img, target_img, float(max_target_val)).mean()))
        else:  # torchmetrics crops every window away: the mean of nothing
            metric.ssim = torch.tensor(float("nan"))
        if self.lpips is not None:
            p = (2 * (pred_img - min_target_val) / rng - 1).expand(-1, 3, -1, -1)
            t = (2 * (target_img - min_target_val) / rng - 1).expand(-1, 3, -1, -1)
            metric.lpips = self.lpips.to(p.device)(in0=p, in1=t).mean()
        return metric


def psnr(pred_img, target_img, data_range):
    """PSNR of one image (or the mean over a leading batch) with the reference's formula
    (den_image_error; no range check on the targets -- bench.py's teacher renders may exceed it)."""
    if not data_range > 0:
        return float("nan")
    t = target_img if target_img.dim() == 4 else target_img.reshape((4 - target_img.dim()) * (1,) + tuple(target_img.shape))
    p = pred_img.reshape(t.shape)
    err = _native.image_error(p, t).cpu()
    pix = t[0].numel()
    vals = [10.0 * math.log10(data_range ** 2 / (float(e) / pix)) if float(e) > 0 else math.inf for e in err[:, 0]]
    return sum(vals) / len(vals)
