"""Import the read-only reference (SimingShan/red-diffeq) IN THIS CONTAINER ONLY, to generate
golden fixtures.  Never imported by tests, bench.py or smoke(): /root/reference does not exist on
the GPU box.

The reference's package ``__init__`` pulls in third-party modules that are not installed here
(``ml_collections``, ``denoising_diffusion_pytorch``, ``ema_pytorch``, ``torchvision``).  They are
replaced by minimal stubs.  The only stub that carries arithmetic on the inversion path is
``denoising_diffusion_pytorch.attend.Attend`` (flash=False branch, denoising-diffusion-pytorch
2.1.1, call sites red_diffeq/models/diffusion.py:25,204,216): softmax(q k^T * d^-1/2) v with zero
dropout.  That restatement is the published algorithm; no reference file pins it, so the U-Net
fixtures are "parity unpinned" at exactly that boundary.
"""
import importlib
import sys
import types

REF = "/root/reference"


class _ConfigDict(dict):
    """Tiny ml_collections.ConfigDict stand-in (attribute access + to_dict)."""

    def __init__(self, d=None):
        super().__init__()
        for k, v in (d or {}).items():
            self[k] = _ConfigDict(v) if isinstance(v, dict) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, _ConfigDict) else v) for k, v in self.items()}


def _install_stubs():
    import torch
    from torch import nn, einsum

    class Attend(nn.Module):
        def __init__(self, dropout=0.0, flash=False, scale=None):
            super().__init__()
            self.flash = flash
            self.scale = scale

        def forward(self, q, k, v):
            scale = self.scale if self.scale is not None else q.shape[-1] ** -0.5
            sim = einsum("b h i d, b h j d -> b h i j", q, k) * scale
            attn = sim.softmax(dim=-1)
            return einsum("b h i j, b h j d -> b h i d", attn, v)

    ddp = types.ModuleType("denoising_diffusion_pytorch")
    att = types.ModuleType("denoising_diffusion_pytorch.attend")
    att.Attend = Attend
    fid = types.ModuleType("denoising_diffusion_pytorch.fid_evaluation")
    fid.FIDEvaluation = object
    ver = types.ModuleType("denoising_diffusion_pytorch.version")
    ver.__version__ = "2.1.1"
    ddp.attend, ddp.fid_evaluation, ddp.version = att, fid, ver
    ema = types.ModuleType("ema_pytorch")
    ema.EMA = object
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tvu = types.ModuleType("torchvision.utils")
    tv.transforms, tv.utils = tvt, tvu
    mlc = types.ModuleType("ml_collections")
    mlc.ConfigDict = _ConfigDict
    for name, mod in {
        "denoising_diffusion_pytorch": ddp,
        "denoising_diffusion_pytorch.attend": att,
        "denoising_diffusion_pytorch.fid_evaluation": fid,
        "denoising_diffusion_pytorch.version": ver,
        "ema_pytorch": ema,
        "torchvision": tv,
        "torchvision.transforms": tvt,
        "torchvision.utils": tvu,
        "ml_collections": mlc,
    }.items():
        sys.modules.setdefault(name, mod)


def load_reference():
    """Return a namespace with the reference modules used by the fixture generators."""
    _install_stubs()
    pkg = types.ModuleType("red_diffeq")
    pkg.__path__ = [REF + "/red_diffeq"]
    sys.modules["red_diffeq"] = pkg
    ns = types.SimpleNamespace()
    ns.pde = importlib.import_module("red_diffeq.solvers.pde")
    ns.inversion = importlib.import_module("red_diffeq.core.inversion")
    ns.losses = importlib.import_module("red_diffeq.core.losses")
    ns.metrics = importlib.import_module("red_diffeq.core.metrics")
    ns.diffusion = importlib.import_module("red_diffeq.models.diffusion")
    ns.reg_diffusion = importlib.import_module("red_diffeq.regularization.diffusion")
    ns.reg_bench = importlib.import_module("red_diffeq.regularization.benchmark")
    ns.reg_base = importlib.import_module("red_diffeq.regularization.base")
    ns.data_trans = importlib.import_module("red_diffeq.utils.data_trans")
    ns.ssim = importlib.import_module("red_diffeq.utils.ssim")
    return ns
