from . import nerf  # noqa: F401
