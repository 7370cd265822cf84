"""Test-only loader for the read-only reference package at /root/reference.

Used ONLY by ``tests/golden/make_golden.py`` (run in the build container, never
on the GPU box) to execute the reference's own pure-PyTorch modules and record
their outputs as golden fixtures.  Nothing in the product package imports this.

The reference package root (``deblur_e_nerf/__init__.py``) imports
pytorch_lightning, which is absent here, so sub-packages are registered as bare
namespace modules whose ``__path__`` points into the reference tree.  Third-party
modules the reference imports get stand-ins:

* ``easydict.EasyDict``: a dict with recursive attribute access (exercised);
* ``nerfacc``: the CPU restatement of nerfacc 0.3.1 in ``oracle/nerfacc.py``
  (ray_marching, OccupancyGrid, render_weight_from_density,
  accumulate_along_rays, ContractionType) -- exercised by the render fixtures,
  which therefore pin the reference's glue around nerfacc, not nerfacc itself;
* ``roma``: the CPU restatement of RoMa 1.2.7 in ``oracle/roma.py`` (exercised by
  the trajectory fixture);
* ``pytorch_lightning``: ``LightningModule`` = ``torch.nn.Module`` (the
  DeblurENeRF fixture binds the reference's methods to a plain module);
* ``pypose``: the CPU restatement of pypose 0.6.7's optimizer base in ``oracle/pypose.py`` (exercised
  by the evaluation fixtures, whose black-level refinement runs the reference's own
  external/optimizer.py subclasses on it);
* ``torchmetrics``: the CPU restatement of torchmetrics 0.6.2's psnr / ssim in ``oracle/metrics.py``;
* ``lpips``: ``LPIPS`` returns zeros (no pretrained network exists offline; the fixtures record no
  LPIPS values);
* ``cv2``: attributes are filled by the fixture that uses them (``make_golden.install_cv2``: imread
  returns the exact samples the fixture wrote, cvtColor restates OpenCV's conversions); otherwise
  import-only; ``tinycudann``: import-only; ``tqdm`` is the real package when importable (the dataset
  queueing fixture runs datasets.py's loops, which call it), else import-only too.
"""
import importlib
import os
import sys
import types

REF_ROOT = "/root/reference"
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _EasyDict(dict):
    """dict with recursive attribute access (what loss.py uses of easydict)."""

    def __init__(self, d=None, **kw):
        super().__init__()
        d = dict(d or {}, **kw)
        for k, v in d.items():
            self[k] = v

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, _EasyDict):
            v = _EasyDict(v)
        super().__setitem__(k, v)

    __setattr__ = __setitem__

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def install():
    if "deblur_e_nerf.models" in sys.modules:
        return
    if not os.path.isdir(REF_ROOT):
        raise RuntimeError("reference tree not present: golden generation only runs in the build container")
    if REPO_ROOT not in sys.path:
        sys.path.insert(0, REPO_ROOT)
    from oracle import metrics as ometrics
    from oracle import nerfacc as onerfacc
    from oracle import pypose as opypose
    from oracle import roma as oroma
    ed = types.ModuleType("easydict")
    ed.EasyDict = _EasyDict
    sys.modules["easydict"] = ed
    try:  # the real progress bar when the image has it (datasets.py's queueing loops call tqdm.tqdm)
        import tqdm  # noqa: F401
    except ImportError:
        pass
    for name in ("cv2", "tqdm", "tinycudann"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["roma"] = oroma.as_module()
    sys.modules["pypose"] = opypose.as_module()
    sys.modules["torchmetrics"] = ometrics.as_module()
    lp = types.ModuleType("lpips")
    import torch

    class LPIPS(torch.nn.Module):
        def __init__(self, net=None):
            super().__init__()
            self.net = net

        def forward(self, in0, in1):
            return torch.zeros(in0.shape[0], 1, 1, 1, dtype=in0.dtype)

    lp.LPIPS = LPIPS
    sys.modules["lpips"] = lp
    pl = types.ModuleType("pytorch_lightning")
    pl.LightningModule = torch.nn.Module
    sys.modules["pytorch_lightning"] = pl
    nf = types.ModuleType("nerfacc")
    for fn in ("ContractionType", "OccupancyGrid", "ray_marching", "render_weight_from_density",
               "render_weight_from_alpha", "accumulate_along_rays"):
        setattr(nf, fn, getattr(onerfacc, fn))
    sys.modules["nerfacc"] = nf
    pkg_root = os.path.join(REF_ROOT, "deblur_e_nerf")
    root = types.ModuleType("deblur_e_nerf")
    root.__path__ = [pkg_root]
    sys.modules["deblur_e_nerf"] = root
    for sub in ("models", "utils", "data", "external", "loss_metric"):
        m = types.ModuleType("deblur_e_nerf." + sub)
        m.__path__ = [os.path.join(pkg_root, sub)]
        sys.modules["deblur_e_nerf." + sub] = m
        setattr(root, sub, m)


def load(modname):
    install()
    return importlib.import_module("deblur_e_nerf." + modname)
