"""OffsetGammaCorrection -- mirror of the reference's evaluation model (models/offset_gamma_correction.py:
4-167): corrected = const_scale * (scale * input^gamma - offset), fitted by the evaluation's
black-level refinement (deblur_e_nerf.py:842-935, external/optimizer.py).

Same constructor, buffer and parameter names (``const_scale``, ``scale``, ``gamma``, ``offset``) and
the same ``forward`` / ``dense_jacobian`` / ``param_jacobian`` / ``jacobian`` contracts.  Shapes (as the
reference supports): const_scale (B, 1, 1, 1, 1), scale / gamma / offset (1 or C, 1, 1, 1), input
(B, C, H, W, R).  This is the evaluation's CPU float64 correction (the reference moves it to the CPU,
:713-716), not part of the training step.
"""
import torch


def _as_tensor(v):
    return v.detach().clone() if torch.is_tensor(v) else torch.tensor(v)


class OffsetGammaCorrection(torch.nn.Module):
    def __init__(self, const_scale=1.0, init_scale=1.0, init_gamma=1.0, init_offset=0.0):
        super().__init__()
        self.register_buffer("const_scale", _as_tensor(const_scale), persistent=False)
        self.scale = torch.nn.Parameter(_as_tensor(init_scale))
        self.gamma = torch.nn.Parameter(_as_tensor(init_gamma))
        self.offset = torch.nn.Parameter(_as_tensor(init_offset))

    def forward(self, input):
        return self.const_scale * (self.scale * input.pow(self.gamma) - self.offset)

    def dense_jacobian(self, input):
        """d output / d (scale, gamma, offset) of each output element w.r.t. the parameter entry
        that element uses: three (B, C, H, W, R) tensors."""
        d_scale = self.const_scale * input.pow(self.gamma)
        d_gamma = self.scale * input.log() * d_scale
        d_offset = (-self.const_scale).expand(input.shape)
        return d_scale, d_gamma, d_offset

    def _check(self, input):
        assert len(self.const_scale) == self.const_scale.numel() == len(input)
        C = input.shape[1]
        for p in (self.scale, self.gamma, self.offset):
            assert len(p) == p.numel() and len(p) in (1, C)
        return C

    @staticmethod
    def _expand_channels(dense, n, C):
        """(B, C, H, W, R) -> (B, C, H, W, R, n, 1, 1, 1): a shared parameter (n = 1) is a plain
        view; a per-channel one (n = C) puts channel c's derivative in column c, zeros elsewhere."""
        if n == 1:
            return dense.reshape(*dense.shape, 1, 1, 1, 1)
        out = dense.new_zeros(*dense.shape, n, 1, 1, 1)
        for c in range(C):
            out[:, c, ..., c, 0, 0, 0] = dense[:, c]
        return out

    def param_jacobian(self, input):
        """The per-parameter (sparse) jacobians, [[d/d scale, d/d gamma, d/d offset]], each
        (B, C, H, W, R, *param.shape)."""
        C = self._check(input)
        dense = self.dense_jacobian(input)
        return [[self._expand_channels(d, len(p), C) for d, p in zip(dense, (self.scale, self.gamma, self.offset))]]

    def jacobian(self, input):
        """The flattened jacobian [J], J (N, S + G + O) with N = input.numel() rows in input order and
        columns scale | gamma | offset (one per parameter entry)."""
        C = self._check(input)
        dense = self.dense_jacobian(input)
        cols = []
        for d, p in zip(dense, (self.scale, self.gamma, self.offset)):
            n = len(p)
            if n == 1:
                cols.append(d.reshape(-1, 1))
            else:
                block = d.new_zeros(*input.shape, n)
                for c in range(C):
                    block[:, c, ..., c] = d[:, c]
                cols.append(block.reshape(-1, n))
        return [torch.cat(cols, dim=1)]
