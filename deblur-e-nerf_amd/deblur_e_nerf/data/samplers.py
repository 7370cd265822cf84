"""Normalized-sample generators of the training batch -- the reference's data/samplers.py
(:4-69): endless iterable datasets yielding one tensor of ``size`` per step.

* ``UniformSampler``  U[low, high)                    (diff / subdiff start positions)
* ``TriangularSampler`` triangular(low, mode, high) by inverse CDF (subdiff lengths, mode 0)
* ``DiracDeltaSampler`` a constant tensor              (diff lengths = 1, interval generators = 0.5)

``size`` is read at every draw: ``DeblurENeRF.update_train_batch_size`` replaces it between
steps (deblur_e_nerf.py:1293-1308).  Host-side RNG (the per-rank ``torch.Generator`` of
DataModule.setup) feeding the HIP path; the draws themselves are tiny CPU tensors.
"""
import torch


class _Sampler(torch.utils.data.IterableDataset):
    def __init__(self, size, dtype=None, generator=None):
        super().__init__()
        self.size = size
        self.dtype = dtype
        self.generator = generator

    def _shape(self):
        return (self.size,) if isinstance(self.size, int) else tuple(self.size)

    def draw(self):
        raise NotImplementedError

    def __iter__(self):
        while True:
            yield self.draw()


class UniformSampler(_Sampler):
    def __init__(self, low, high, size, dtype=None, generator=None):
        super().__init__(size, dtype, generator)
        self.low, self.high = low, high

    def draw(self):
        u = torch.rand(self._shape(), dtype=self.dtype, generator=self.generator)
        return u * (self.high - self.low) + self.low


class TriangularSampler(_Sampler):
    """Inverse-CDF sampling of the triangular distribution on [low, high] with peak at mode."""

    def __init__(self, low, high, size, mode, dtype=None, generator=None):
        super().__init__(size, dtype, generator)
        if not all(isinstance(v, (int, float)) for v in (low, high, mode)) or not low <= mode <= high:
            raise ValueError("TriangularSampler needs numbers low <= mode <= high")
        self.low, self.high, self.mode = low, high, mode
        span = high - low
        self.mode_cum_prob = (mode - low) / span  # F(mode)
        self.k1 = span * (mode - low)
        self.k2 = span * (high - mode)

    def draw(self):
        u = torch.rand(self._shape(), dtype=self.dtype, generator=self.generator)
        left = self.low + torch.sqrt(u * self.k1)
        right = self.high - torch.sqrt((1 - u) * self.k2)
        return torch.where(u <= self.mode_cum_prob, left, right)


class DiracDeltaSampler(_Sampler):
    def __init__(self, center, size, dtype=None):
        super().__init__(size, dtype)
        self.center = center

    def draw(self):
        return torch.full(self._shape(), self.center, dtype=self.dtype)


__all__ = ["UniformSampler", "TriangularSampler", "DiracDeltaSampler"]
