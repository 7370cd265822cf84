from . import datamodule, datasets, samplers  # noqa: F401
