"""Oracle: the pypose 0.6.7 optimizer base the reference's external/optimizer.py subclasses -- CPU
restatement (test infrastructure only, see oracle/__init__.py).

pypose (environment.yml:30, pip pypose==0.6.7) is not installed here (no network).  The reference
subclasses ``pp.optim.GaussNewton`` / ``pp.optim.LevenbergMarquardt`` (external/optimizer.py:19-111)
and overrides ``step``, so what it takes from pypose is the constructor state and helpers that
``step`` reads, restated from pypose's published source (pypose/optim/optimizer.py, solver.py,
strategy.py, kernel.py, corrector.py):

* ``RobustModel``: ``forward(input, target)`` -> (model(input) - target,); ``loss`` = sum over
  residuals of kernel(r.square().sum(-1)).sum() with the Trivial (identity) kernel;
  ``normalize_RWJ`` concatenates the flattened residuals and the jacobian rows;
* ``_Optimizer.update_parameter``: the step split by parameter sizes, added in registration order;
* ``GaussNewton(model, solver=LSTSQ())``: weight None, Trivial corrector;
* ``LevenbergMarquardt(model, strategy=TrustRegion(...), reject=16, min=1e-6, max=1e32)``: the
  Cholesky solver, param-group defaults {min, max} + the strategy's (with damping = 1 / radius);
* ``TrustRegion.update``: quality = (last - loss) / -(J D)^T (2 R + J D); radius x up above
  ``high``, kept above ``low``, else x down and down x factor; radius clamped to [min, max];
  damping = 1 / radius.

Parity of this restatement against pypose itself is UNPINNED.  It stands in for pypose when
tests/golden/make_golden.py runs the reference's evaluation_epoch_end, whose own logic (the affine
fit, the warm start, the early stop, the effective parameters, the metric loop) is what the
``eval_epoch_*`` fixtures pin.
"""
import types

import torch


class Trivial(torch.nn.Module):
    def forward(self, x, J=None, R=None):
        return x if J is None else (R, J)


class _TrivialCorrector(torch.nn.Module):
    def forward(self, R, J):
        return R, J


class RobustModel(torch.nn.Module):
    def __init__(self, model, kernel=None):
        super().__init__()
        self.model = model
        self.kernel = [Trivial()] if kernel is None else kernel

    def model_forward(self, input):
        return self.model(*input) if isinstance(input, tuple) else self.model(input)

    def residual(self, output, target):
        return output if target is None else output - target

    def forward(self, input, target):
        return (self.residual(self.model_forward(input), target),)

    def loss(self, input, target):
        residuals = self.forward(input, target)
        return sum(self.kernel[0](r.square().sum(-1)).sum() for r in residuals)

    def normalize_RWJ(self, R, weight, J):
        assert weight is None
        R = torch.cat([r.reshape(-1) for r in R])
        J = torch.cat(list(J)) if isinstance(J, (tuple, list)) else J
        return R, None, J


class LSTSQ(torch.nn.Module):
    def __init__(self, rcond=None, driver=None):
        super().__init__()
        self.rcond, self.driver = rcond, driver

    def forward(self, A, b):
        x = torch.linalg.lstsq(A, b, rcond=self.rcond, driver=self.driver).solution
        assert not torch.any(torch.isnan(x)), "linear solver returned NaN"
        return x


class Cholesky(torch.nn.Module):
    def __init__(self, upper=False):
        super().__init__()
        self.upper = upper

    def forward(self, A, b):
        L, _ = torch.linalg.cholesky_ex(A, upper=self.upper)
        assert not torch.any(torch.isnan(L)), "Cholesky decomposition failed"
        return torch.cholesky_solve(b, L, upper=self.upper)


class TrustRegion:
    def __init__(self, radius=1e6, high=0.5, low=1e-3, up=2.0, down=0.5, factor=4.0, min=1e-6, max=1e16):
        self.defaults = {"radius": radius, "high": high, "low": low, "up": up, "down": down, "factor": factor,
                         "damping": 1.0 / radius}
        self.min, self.max, self.down = min, max, down

    def update(self, pg, last, loss, J, D, R, *args, **kwargs):
        JD = J @ D
        quality = (last - loss) / -((JD).mT @ (2 * R + JD)).squeeze()
        pg["radius"] = 1.0 / pg["damping"]
        if quality > pg["high"]:
            pg["radius"] = pg["up"] * pg["radius"]
            pg["down"] = self.down
        elif quality > pg["low"]:
            pg["down"] = self.down
        else:
            pg["radius"] = pg["radius"] * pg["down"]
            pg["down"] = pg["down"] * pg["factor"]
        pg["radius"] = max(self.min, min(float(pg["radius"]), self.max))
        pg["damping"] = 1.0 / pg["radius"]


class _Optimizer(torch.optim.Optimizer):
    def update_parameter(self, params, step):
        steps = step.split([p.numel() for p in params if p.requires_grad])
        for p, d in zip([p for p in params if p.requires_grad], steps):
            p.add_(d.view(p.shape))


class GaussNewton(_Optimizer):
    def __init__(self, model, solver=None, kernel=None, corrector=None, weight=None, vectorize=True):
        super().__init__(model.parameters(), defaults={})
        self.solver = LSTSQ() if solver is None else solver
        self.jackwargs = {"vectorize": vectorize, "flatten": False}
        self.weight = weight
        self.corrector = [_TrivialCorrector()] if corrector is None else corrector
        self.model = RobustModel(model, kernel)


class LevenbergMarquardt(_Optimizer):
    def __init__(self, model, solver=None, strategy=None, kernel=None, corrector=None, weight=None, reject=16,
                 min=1e-6, max=1e32, vectorize=True):
        self.strategy = TrustRegion() if strategy is None else strategy
        defaults = {"min": min, "max": max, **self.strategy.defaults}
        super().__init__(model.parameters(), defaults=defaults)
        self.solver = Cholesky() if solver is None else solver
        self.jackwargs = {"vectorize": vectorize, "flatten": False}
        self.reject, self.reject_count = reject, 0
        self.weight = weight
        self.corrector = [_TrivialCorrector()] if corrector is None else corrector
        self.model = RobustModel(model, kernel)


def as_module():
    """A ``pypose`` module object with what the reference touches: pp.optim.{GaussNewton,
    LevenbergMarquardt}, pp.optim.solver.{LSTSQ, Cholesky}, pp.optim.strategy.TrustRegion."""
    pp = types.ModuleType("pypose")
    optim = types.ModuleType("pypose.optim")
    optim.GaussNewton, optim.LevenbergMarquardt = GaussNewton, LevenbergMarquardt
    optim.solver = types.SimpleNamespace(LSTSQ=LSTSQ, Cholesky=Cholesky)
    optim.strategy = types.SimpleNamespace(TrustRegion=TrustRegion)
    optim.functional = types.SimpleNamespace()
    pp.optim = optim
    return pp
