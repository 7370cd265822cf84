"""Adam on libden.so -- the optimizer of DeblurENeRF.configure_optimizers
(deblur_e_nerf.py:1055-1112: torch.optim.Adam with per-group lr / weight decay).

``Adam`` is a ``torch.optim.Optimizer`` with torch.optim.Adam's semantics (amsgrad off, L2
weight decay added to the gradient, bias corrections formed in double and rounded like torch's
scalars) whose update runs in den_adam_step / den_adam_step_f64.  A parameter group whose
parameters are consecutive views of one flat buffer (the MLP: VanillaNeRFRadianceField keeps
its 24 tensors in one buffer, and their gradients arrive as views of one flat gradient) is
stepped with ONE launch over the whole buffer.  MultiStepLR and other schedulers work
unchanged (they edit ``group['lr']``).

State lives in ``self.state[p]`` with torch.optim.Adam's keys (``step`` a CPU float tensor,
``exp_avg``, ``exp_avg_sq``), so ``state_dict()`` / ``load_state_dict()`` round-trip and are
interchangeable with torch.optim.Adam checkpoints.  For a flat group the per-parameter moments
are views of one flat moment buffer; after a load (which hands back separate tensors) the
buffer is rebuilt from them on the next step.
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


def _new_step():
    return torch.tensor(0.0, dtype=torch.float32)


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyperparameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    def _flat_moments(self, params, flat_p):
        """(exp_avg, exp_avg_sq, step) flat buffers over the group, each param's state a view of
        them; None when the params' states disagree on the step (mixed history)."""
        states = [self.state[p] for p in params]
        steps = {float(s["step"]) for s in states if s}
        if len(steps) > 1 or (steps and not all(states)):
            return None
        step = steps.pop() if steps else 0.0
        if all(states):
            ea = _flat_span([s["exp_avg"] for s in states])
            eas = _flat_span([s["exp_avg_sq"] for s in states])
            if (ea is not None and eas is not None and ea.numel() == flat_p.numel()
                    and eas.numel() == flat_p.numel() and ea.device == flat_p.device):
                return ea, eas, step
        # (re)build the flat buffers, keeping any loaded moments
        ea, eas = torch.zeros_like(flat_p), torch.zeros_like(flat_p)
        pos = 0
        for p, s in zip(params, states):
            n = p.numel()
            va, vs = ea[pos:pos + n].view_as(p), eas[pos:pos + n].view_as(p)
            if s:
                va.copy_(s["exp_avg"])
                vs.copy_(s["exp_avg_sq"])
            s.update(step=s.get("step", _new_step()), exp_avg=va, exp_avg_sq=vs)
            pos += n
        return ea, eas, step

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
            fm = self._flat_moments(params, flat_p) if flat_g is not None else None
            if fm is not None:
                ea, eas, step = fm
                step = int(step) + 1
                for p in params:
                    self.state[p]["step"].fill_(float(step))
                _native.adam_step(flat_p, flat_g, ea, eas, *args, step)
                continue
            for p in params:
                st = self.state[p]
                if not st:
                    st.update(step=_new_step(), exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p))
                st["step"] += 1
                for k in ("exp_avg", "exp_avg_sq"):
                    if not st[k].is_contiguous():
                        st[k] = st[k].contiguous()
                _native.adam_step(p.view(-1) if p.is_contiguous() else p, p.grad.contiguous().view(-1),
                                  st["exp_avg"].view(-1), st["exp_avg_sq"].view(-1), *args, int(st["step"]))
        return loss
