"""TV / Tikhonov regularisers (reference red_diffeq/regularization/benchmark.py:4-37) on the
HIP smooth-regulariser kernel (K6).  Computed on the padded (B,1,72,72) model, pad included,
exactly like the reference."""
import torch

from .. import _hip

_TV, _L2 = 0, 1


class _SmoothReg(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, kind):
        _hip.require_device(mu)
        if mu.dim() != 4 or mu.shape[1] != 1:
            raise ValueError(f"expected (B,1,H,W), got {tuple(mu.shape)}")
        m = mu.float().contiguous()
        B, _, H, W = m.shape
        loss = torch.empty(B, dtype=torch.float32, device=m.device)
        _hip.check(_hip.lib().rdq_smooth_reg_forward(kind, B, H, W, _hip.ptr(m), _hip.ptr(loss),
                                                     _hip.stream_of(m)), "rdq_smooth_reg_forward")
        ctx.save_for_backward(m)
        ctx.kind = kind
        return loss

    @staticmethod
    def backward(ctx, gout):
        (m,) = ctx.saved_tensors
        B, _, H, W = m.shape
        grad = torch.empty_like(m)
        gout = gout.float().contiguous()
        _hip.check(_hip.lib().rdq_smooth_reg_backward(ctx.kind, B, H, W, _hip.ptr(m), _hip.ptr(gout),
                                                      _hip.ptr(grad), _hip.stream_of(m)),
                   "rdq_smooth_reg_backward")
        return grad, None


def total_variation_loss(mu: torch.Tensor) -> torch.Tensor:
    """mean|d/dx| + mean|d/dz| per model (benchmark.py:4-19)."""
    return _SmoothReg.apply(mu, _TV)


def tikhonov_loss(mu: torch.Tensor) -> torch.Tensor:
    """mean (d/dx)^2 + mean (d/dz)^2 per model (benchmark.py:22-37)."""
    return _SmoothReg.apply(mu, _L2)
