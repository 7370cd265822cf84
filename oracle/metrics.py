"""Oracle: the torchmetrics 0.6.2 image metrics the reference's Metric calls -- CPU restatement (test
infrastructure only, see oracle/__init__.py).

torchmetrics (environment.yml:21, torchmetrics=0.6.2) is not installed here.  The reference calls
(loss_metric/metric.py:68-81):

* ``psnr(preds, target, data_range, reduction="elementwise_mean", dim=(1, 2, 3))``: per image the
  sum of squared errors over ``dim`` and its count, psnr = (2 ln(data_range) - ln(sse / n)) x
  10 / ln(10) with data_range as an f32 tensor, mean over the images;
* ``ssim(preds, target, data_range, reduction="elementwise_mean")``: an 11 x 11 Gaussian kernel
  (sigma 1.5; the 1-D gaussian over arange(-5, 6), normalised, and its outer product, in the inputs'
  dtype), c1 = (0.01 range)^2, c2 = (0.03 range)^2; preds / target reflect-padded by 5; one grouped
  conv2d of [p, t, p^2, t^2, p t]; mu / sigma / the SSIM index; the index cropped by 5 on every side;
  the mean of what remains.

Parity of this restatement against torchmetrics itself is UNPINNED (restated from its published
0.6.2 source).  It stands in for torchmetrics when tests/golden/make_golden.py runs the reference's
Metric and is the checker of den_ssim.
"""
import math
import types

import torch
import torch.nn.functional as F


def psnr(preds, target, data_range=None, base=10.0, reduction="elementwise_mean", dim=None):
    assert dim is not None and reduction == "elementwise_mean"
    dr = torch.tensor(float(data_range))
    sse = torch.sum((preds - target) ** 2, dim=dim)
    n = torch.tensor(math.prod(preds.shape[d] for d in dim), device=sse.device)
    vals = (2 * torch.log(dr) - torch.log(sse / n)) * (10 / torch.log(torch.tensor(base)))
    return vals.mean()


def _gaussian(kernel_size, sigma, dtype):
    dist = torch.arange((1 - kernel_size) / 2, (1 + kernel_size) / 2, 1, dtype=dtype)
    gauss = torch.exp(-torch.pow(dist / sigma, 2) / 2)
    return (gauss / gauss.sum()).unsqueeze(dim=0)


def ssim_map(preds, target, data_range, kernel_size=(11, 11), sigma=(1.5, 1.5), k1=0.01, k2=0.03):
    """The cropped SSIM index map (B, C, H - 10, W - 10)."""
    c1 = pow(k1 * data_range, 2)
    c2 = pow(k2 * data_range, 2)
    channel = preds.size(1)
    gx = _gaussian(kernel_size[0], sigma[0], preds.dtype)
    gy = _gaussian(kernel_size[1], sigma[1], preds.dtype)
    kernel = torch.matmul(gx.t(), gy).expand(channel, 1, kernel_size[0], kernel_size[1])
    ph, pw = (kernel_size[0] - 1) // 2, (kernel_size[1] - 1) // 2
    preds = F.pad(preds, (ph, ph, pw, pw), mode="reflect")
    target = F.pad(target, (ph, ph, pw, pw), mode="reflect")
    inputs = torch.cat((preds, target, preds * preds, target * target, preds * target))
    outputs = F.conv2d(inputs, kernel, groups=channel)
    B = preds.size(0)
    o = [outputs[x * B:(x + 1) * B] for x in range(len(outputs) // B)]
    mu_pp, mu_tt, mu_pt = o[0].pow(2), o[1].pow(2), o[0] * o[1]
    s_pp, s_tt, s_pt = o[2] - mu_pp, o[3] - mu_tt, o[4] - mu_pt
    upper = 2 * s_pt + c2
    lower = s_pp + s_tt + c2
    idx = ((2 * mu_pt + c1) * upper) / ((mu_pp + mu_tt + c1) * lower)
    return idx[..., ph:-ph, pw:-pw]


def ssim(preds, target, data_range=None, reduction="elementwise_mean"):
    assert reduction == "elementwise_mean"
    return ssim_map(preds, target, data_range).mean()


def as_module():
    """A ``torchmetrics`` module object with ``functional.psnr`` / ``functional.ssim``."""
    tm = types.ModuleType("torchmetrics")
    tm.functional = types.SimpleNamespace(psnr=psnr, ssim=ssim)
    return tm
