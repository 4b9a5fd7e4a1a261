import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "red-diffeq_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

collect_ignore_glob = ["golden/*.py"]   # fixture generators: run the reference, never on the box


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")


def record_margin(test, case, measured, bar):
    """One parity test's measured value against its bar, appended as a JSON line to
    $RDQ_EVIDENCE_DIR/margins.jsonl (GPU evidence runs: profiles/r*/margins.jsonl), so every bar can
    be read next to what the kernels actually achieve.  No-op without the variable."""
    import json
    d = os.environ.get("RDQ_EVIDENCE_DIR")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    rec = {"test": test, "case": str(case), "measured": float(measured), "bar": float(bar),
           "ratio": float(measured) / float(bar) if bar else None}
    with open(os.path.join(d, "margins.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def ctx_of(z):
    return {k[4:]: (z[k].item() if z[k].ndim == 0 else z[k]) for k in z.files if k.startswith("ctx_")}


def vnorm(v):
    return ((v - 1500) / 3000 * 2 - 1).astype(np.float32)


def regenerate_draws(rows, randn_shape):
    """The reference's global-RNG draws of a long trajectory (tests/golden/make_long.py), re-made
    from torch's CPU generator (seed 1234, as the fixture run) in call order: rows of (kind 0 randn /
    1 randint, low, high, numel, float64 sum); every draw is checked against its recorded sum."""
    import torch
    g = torch.Generator().manual_seed(1234)
    out = []
    for kind, low, high, n, s in rows:
        if kind == 0:
            assert n == int(np.prod(randn_shape)), (n, randn_shape)
            d = torch.randn(randn_shape, generator=g)
            name = "randn"
        else:
            d = torch.randint(int(low), int(high), (int(n),), generator=g)
            name = "randint"
        assert float(d.double().sum()) == s, ("regenerated draw differs from the reference's", len(out))
        out.append((name, d.numpy()))
    return out


class replay_draws:
    """Replay the reference's recorded global-RNG draws (tests/golden/make_golden.py:record_draws)
    in call order: inside the block every torch.randn / rand / randint / randperm call returns the
    next recorded array on the requested device.  The kind and shape of each call are checked, so
    a product path that draws in a different order, or draws more or fewer times, fails."""

    FNS = ("randn", "rand", "randint", "randperm")

    def __init__(self, z, randn_shape=(1, 1, 72, 72)):
        import torch
        self.torch = torch
        if "draw_rows" in z.files:
            self.queue = regenerate_draws(z["draw_rows"], randn_shape)
        else:
            kinds = [str(k) for k in z["draw_kinds"]] if "draw_kinds" in z.files else []
            self.queue = [(k, z[f"draw{i}"]) for i, k in enumerate(kinds)]
        self.pos = 0

    @staticmethod
    def _shape(name, args, kw):
        if name == "randperm":
            return (int(args[0]),)
        if name == "randint":
            size = kw.get("size", args[-1] if args and isinstance(args[-1], (tuple, list)) else None)
            return tuple(int(s) for s in size)
        size = args[0] if len(args) == 1 and not isinstance(args[0], int) else args
        return tuple(int(s) for s in (kw.get("size") or size))

    def _fn(self, name):
        def draw(*args, **kw):
            assert self.pos < len(self.queue), f"unrecorded torch.{name} call #{self.pos}"
            kind, val = self.queue[self.pos]
            assert kind == name, f"draw #{self.pos}: product called torch.{name}, reference {kind}"
            assert self._shape(name, args, kw) == val.shape, (name, self._shape(name, args, kw), val.shape)
            self.pos += 1
            t = self.torch.from_numpy(val.copy())
            if kw.get("dtype") is not None:
                t = t.to(kw["dtype"])
            return t.to(kw["device"]) if kw.get("device") is not None else t
        return draw

    def __enter__(self):
        self.orig = {n: getattr(self.torch, n) for n in self.FNS}
        for n in self.FNS:
            setattr(self.torch, n, self._fn(n))
        return self

    def __exit__(self, *exc):
        for n, f in self.orig.items():
            setattr(self.torch, n, f)
        if exc[0] is None:
            assert self.pos == len(self.queue), f"{len(self.queue) - self.pos} recorded draws not consumed"


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
