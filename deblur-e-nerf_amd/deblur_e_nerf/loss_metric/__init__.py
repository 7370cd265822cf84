from . import loss, metric  # noqa: F401
