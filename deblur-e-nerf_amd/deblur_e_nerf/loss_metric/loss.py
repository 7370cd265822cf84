"""Event losses -- mirror of the reference's loss_metric/loss.py (Loss, :6-96).

Same constructor ``Loss(loss_weight, loss_error_fn, loss_normalize)``, the same
``compute(batch_event, batch_diff=None, batch_subdiff=None, mean_contrast_threshold=None)
-> EasyDict(log_intensity_diff=..., log_intensity_tv=...)`` and the same masked means:

* diff: mean over ``batch_diff.is_valid`` of err(Δ̂ / c, f32(ts_diff * (lid / (end - start)) / c))
* TV:   mean over ``batch_subdiff.is_valid`` of err(Δ̂_sub / c, 0)

with c the mean contrast threshold when normalised, else 1.  The target (f64 arithmetic rounded
to f32) and the masked means with their gradients run in libden.so (den_event_target /
den_event_target_bwd, den_event_loss_fwd / _bwd); gradients reach Δ̂, the contrast thresholds
(through lid and c) and the event timestamps.  An empty valid set gives NaN, as torch's empty
mean does.
"""
import torch

from .. import _native
from ..utils.easydict import EasyDict


class Loss(torch.nn.Module):
    LOSS_NAMES = ["log_intensity_diff", "log_intensity_tv"]
    ERROR_FNS = ("l1", "mse", "huber", "mape")

    def __init__(self, loss_weight, loss_error_fn, loss_normalize):
        super().__init__()
        assert set(self.LOSS_NAMES) <= set(loss_weight.keys())
        for v in loss_weight.values():
            assert isinstance(v, (int, float)) and v >= 0
        assert sum(loss_weight.values()) > 0
        self.loss_weight = EasyDict(loss_weight)
        self.error_fn = EasyDict()
        for key in self.LOSS_NAMES:
            fn = loss_error_fn[key]
            if fn not in self.ERROR_FNS:
                raise NotImplementedError(f"error function {fn!r}: libden implements l1, mse and huber (delta = 1)")
            self.error_fn[key] = fn
        self.normalize = EasyDict(loss_normalize)

    def compute(self, batch_event, batch_diff=None, batch_subdiff=None, mean_contrast_threshold=None):
        batch_mean_loss = EasyDict({})
        if self.loss_weight.log_intensity_diff > 0:
            batch_mean_loss.log_intensity_diff = self.log_intensity_diff(batch_event, batch_diff,
                                                                         mean_contrast_threshold)
        if self.loss_weight.log_intensity_tv > 0:
            batch_mean_loss.log_intensity_tv = self.log_intensity_tv(batch_subdiff, mean_contrast_threshold)
        return batch_mean_loss

    @staticmethod
    def _const(c, like):
        if c is None or not torch.is_tensor(c):
            return torch.full((1,), 1.0 if c is None else float(c), dtype=torch.float32, device=like.device)
        return c.reshape(1).to(torch.float32)

    def log_intensity_diff(self, batch_event, batch_diff, mean_contrast_threshold):
        c = self._const(mean_contrast_threshold if self.normalize.log_intensity_diff else None,
                        batch_diff.log_intensity_diff)
        target = _native.EventTargetFunction.apply(batch_diff.ts_diff, batch_event.log_intensity_diff,
                                                   batch_event.end_ts, batch_event.start_ts, c)
        return _native.EventLossFunction.apply(batch_diff.log_intensity_diff.float().contiguous(), target, c,
                                               batch_diff.is_valid, self.error_fn.log_intensity_diff)

    def log_intensity_tv(self, batch_subdiff, mean_contrast_threshold):
        c = self._const(mean_contrast_threshold if self.normalize.log_intensity_tv else None,
                        batch_subdiff.log_intensity_diff)
        return _native.EventLossFunction.apply(batch_subdiff.log_intensity_diff.float().contiguous(), None, c,
                                               batch_subdiff.is_valid, self.error_fn.log_intensity_tv)
