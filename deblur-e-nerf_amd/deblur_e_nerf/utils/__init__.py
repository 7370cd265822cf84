from . import modules  # noqa: F401
