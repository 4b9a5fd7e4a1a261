"""TV / Tikhonov regularisers (reference red_diffeq/regularization/benchmark.py:4-37) on the
HIP smooth-regulariser kernel (K6).  Computed on the padded (B,1,72,72) model, pad included,
exactly like the reference."""
import torch

from .. import _hip
from .. import ops  # noqa: F401  (registers torch.ops.red_diffeq.*)

_TV, _L2 = 0, 1


class _SmoothReg(torch.autograd.Function):
    """torch.ops.red_diffeq.smooth_reg / smooth_reg_backward (K6)."""

    @staticmethod
    def forward(ctx, mu, kind):
        _hip.require_device(mu)
        if mu.dim() != 4 or mu.shape[1] != 1:
            raise ValueError(f"expected (B,1,H,W), got {tuple(mu.shape)}")
        ctx.save_for_backward(mu)
        ctx.kind = kind
        return torch.ops.red_diffeq.smooth_reg(mu, kind)

    @staticmethod
    def backward(ctx, gout):
        (mu,) = ctx.saved_tensors
        return torch.ops.red_diffeq.smooth_reg_backward(mu, gout, ctx.kind), None


def total_variation_loss(mu: torch.Tensor) -> torch.Tensor:
    """mean|d/dx| + mean|d/dz| per model (benchmark.py:4-19)."""
    return _SmoothReg.apply(mu, _TV)


def tikhonov_loss(mu: torch.Tensor) -> torch.Tensor:
    """mean (d/dx)^2 + mean (d/dz)^2 per model (benchmark.py:22-37)."""
    return _SmoothReg.apply(mu, _L2)
