"""EasyDict: a dict with recursive attribute access -- the container the reference's
training step, loss and configs use (the third-party ``easydict`` package, absent here).
Nested plain dicts become EasyDicts on assignment, so ``batch.diff.ts_diff = ...`` works as in
the reference (deblur_e_nerf.py:397-549, loss.py:46)."""


class EasyDict(dict):
    def __init__(self, d=None, **kwargs):
        super().__init__()
        for k, v in dict(d or {}, **kwargs).items():
            self[k] = v

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, EasyDict):
            v = EasyDict(v)
        elif isinstance(v, (list, tuple)):
            v = type(v)(EasyDict(x) if isinstance(x, dict) and not isinstance(x, EasyDict) else x for x in v)
        super().__setitem__(k, v)

    def __setattr__(self, k, v):
        self[k] = v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __delattr__(self, k):
        try:
            del self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def update(self, e=None, **f):
        for k, v in dict(e or {}, **f).items():
            self[k] = v

    def pop(self, k, *args):
        return super().pop(k, *args)
