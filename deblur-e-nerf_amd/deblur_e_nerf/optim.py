"""Adam on libden.so -- the optimizer of DeblurENeRF.configure_optimizers
(deblur_e_nerf.py:1055-1112: torch.optim.Adam with per-group lr / weight decay).

``Adam`` is a ``torch.optim.Optimizer`` with torch.optim.Adam's semantics (amsgrad off, L2
weight decay added to the gradient, bias corrections formed in double and rounded like torch's
scalars) whose update runs in den_adam_step / den_adam_step_f64.  A parameter group whose
parameters are consecutive views of one flat buffer (the MLP: VanillaNeRFRadianceField keeps
its 24 tensors in one buffer, and their gradients arrive as views of one flat gradient) is
stepped with ONE launch over the whole buffer.  MultiStepLR and other schedulers work
unchanged (they edit ``group['lr']``).
"""
import torch

from . import _native


def _flat_span(tensors):
    """(base tensor, offset, numel) when the tensors are consecutive views of one contiguous
    buffer, else None."""
    if not tensors:
        return None
    t0 = tensors[0]
    if any(t is None or not t.is_contiguous() or t.dtype != t0.dtype or t.untyped_storage().data_ptr()
           != t0.untyped_storage().data_ptr() for t in tensors):
        return None
    off = t0.storage_offset()
    pos = off
    for t in tensors:
        if t.storage_offset() != pos:
            return None
        pos += t.numel()
    base = torch.empty(0, dtype=t0.dtype, device=t0.device).set_(t0.untyped_storage(), off, (pos - off,))
    return base


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyperparameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._flat_state = {}  # per flat-buffer group: step, exp_avg, exp_avg_sq over the whole buffer

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            b1, b2 = group["betas"]
            args = (group["lr"], b1, b2, group["eps"], group["weight_decay"])
            flat_p = _flat_span(params) if len(params) > 1 else None
            flat_g = _flat_span([p.grad for p in params]) if flat_p is not None else None
            if flat_p is not None and flat_g is not None:
                st = self._flat_state.setdefault(id(group), {})
                if not st or st["exp_avg"].numel() != flat_p.numel():
                    st.update(step=0, exp_avg=torch.zeros_like(flat_p), exp_avg_sq=torch.zeros_like(flat_p))
                st["step"] += 1
                _native.adam_step(flat_p, flat_g, st["exp_avg"], st["exp_avg_sq"], *args, st["step"])
                continue
            for p in params:
                st = self.state[p]
                if not st:
                    st.update(step=0, exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p))
                st["step"] += 1
                _native.adam_step(p.view(-1) if p.is_contiguous() else p, p.grad.contiguous().view(-1),
                                  st["exp_avg"].view(-1), st["exp_avg_sq"].view(-1), *args, st["step"])
        return loss
