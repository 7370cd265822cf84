"""deblur_e_nerf -- MI355X-native (gfx950) hot path of Deblur e-NeRF.

Module paths mirror the reference package (wengflow/deblur-e-nerf):
``deblur_e_nerf.models``, ``deblur_e_nerf.loss_metric``,
``deblur_e_nerf.external``, ``deblur_e_nerf.utils``.  All arithmetic of the
render / event-measurement path runs in libden.so (HIP kernels for gfx950);
see DESIGN.md.
"""
from . import _native  # noqa: F401
from . import data, loss_metric, models, utils  # noqa: F401  (deblur_e_nerf/__init__.py:1)

__version__ = "0.1.0"
