from . import datasets, easydict, modules  # noqa: F401
