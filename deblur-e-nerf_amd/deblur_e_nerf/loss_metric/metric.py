"""Evaluation metrics -- mirror of the reference's loss_metric/metric.py (Metric, :8-92).

Same ``compute(pred_img, target_img, min_target_val, max_target_val) -> EasyDict`` with the
reference's L1 (mean absolute error) and PSNR (torchmetrics.functional.psnr with
``data_range = max - min``, per image over (C, H, W), mean over the batch: 10 log10(range^2 /
MSE)); the per-image error sums run in den_image_error.  SSIM and LPIPS (torchmetrics / lpips
networks, absent here) are not part of the hot path and are left out.
"""
import math

import torch

from .. import _native
from ..utils.easydict import EasyDict


class Metric(torch.nn.Module):
    METRIC_NAMES = ["l1", "psnr"]

    def __init__(self, metric_lpips_net=None):
        super().__init__()
        self.lpips_net = metric_lpips_net

    def init_batch_metric(self):
        return EasyDict({name: [] for name in self.METRIC_NAMES})

    def compute(self, pred_img, target_img, min_target_val, max_target_val):
        assert pred_img.shape == target_img.shape
        assert 2 <= target_img.dim() <= 4
        if target_img.dim() > 2:
            assert target_img.shape[-3] in (1, 3)
        assert 0 <= min_target_val < max_target_val
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
        return metric


def psnr(pred_img, target_img, data_range):
    """PSNR of one image (or the mean over a leading batch) with the reference's formula."""
    m = Metric()
    return float(m.compute(pred_img, target_img, 0.0, float(data_range)).psnr) if data_range > 0 else float("nan")
