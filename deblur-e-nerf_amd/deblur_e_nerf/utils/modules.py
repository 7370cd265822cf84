"""Parametrisations used by the model components (reference utils/modules.py:58-94).

Scalar parameter transforms stay in PyTorch (host glue on a handful of
scalars); they are applied through torch.nn.utils.parametrize exactly as the
reference does, so parameter names (``parametrizations.<name>.original``) and
checkpoints match.
"""
import torch


class Softplus(torch.nn.Module):
    def __init__(self, beta=1, threshold=20):
        super().__init__()
        self.beta = beta
        self.threshold = threshold

    def forward(self, x):
        return torch.nn.functional.softplus(x, self.beta, self.threshold)

    def right_inverse(self, y):
        # inverse softplus, linear above the threshold -- the reference's exact expression
        # (utils/modules.py:67-75), so parametrised originals match it bit for bit
        return torch.where(y * self.beta > self.threshold, y, torch.log(torch.exp(self.beta * y) - 1) / self.beta)


class ScaledShiftedSigmoid(torch.nn.Module):
    """scale * sigmoid(x / scale) + low; keeps sigmoid's gradient profile."""

    def __init__(self, low=0, high=1):
        super().__init__()
        self.low = low
        self.scale = high - low

    def forward(self, x):
        return self.scale * torch.sigmoid(x / self.scale) + self.low

    def right_inverse(self, y):
        return self.scale * torch.logit((y - self.low) / self.scale)


def freeze(module):
    for p in module.parameters():
        p.requires_grad_(False)


def unfreeze(module):
    for p in module.parameters():
        p.requires_grad_(True)


def detach_clone_named_parameters(module):
    """utils/modules.py:38-42: (name, detached copy) of every parameter."""
    return ((name, p.detach().clone()) for name, p in module.named_parameters())


def named_parameters_allclose(module, other_named_parameters):
    """utils/modules.py:45-57: every parameter allclose to its recorded copy."""
    mine, other = dict(module.named_parameters()), dict(other_named_parameters)
    assert mine.keys() == other.keys()
    return all(torch.allclose(mine[k], other[k]) for k in mine)
