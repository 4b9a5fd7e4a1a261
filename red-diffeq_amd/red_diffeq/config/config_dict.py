"""Minimal stand-in for ml_collections.ConfigDict (not installed on the MI355X image).

Supports what red-diffeq uses: attribute + item access, nested dicts, ``to_dict()``, ``get``,
``items()``, ``getattr(cfg, key, default)`` (reference scripts/run_inversion.py:246-248,287).
"""


class ConfigDict(dict):
    def __init__(self, d=None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = v

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, ConfigDict):
            v = ConfigDict(v)
        super().__setitem__(k, v)

    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, ConfigDict) else v) for k, v in self.items()}

    def copy_and_resolve_references(self):
        return ConfigDict(self.to_dict())
