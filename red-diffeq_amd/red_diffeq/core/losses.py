"""LossCalculator (reference red_diffeq/core/losses.py:8-66) on the HIP L1 kernel (K5)."""
from typing import Optional

import torch

from .. import _hip
from ..regularization.base import RegularizationMethod


class _L1Misfit(torch.autograd.Function):
    """Per-model masked L1 misfit: forward rdq_l1_forward, backward rdq_l1_backward
    (dpred = sign(pred - y) * mask * gout / nobs, exactly the autograd of losses.py:27-39)."""

    @staticmethod
    def forward(ctx, pred, y, mask, nobs_override):
        _hip.require_device(pred, y, mask)
        pred = pred.float().contiguous()
        y = y.float().contiguous()
        mask = None if mask is None else mask.float().contiguous()
        B = pred.shape[0]
        n = pred.numel() // B
        L = _hip.lib()
        loss = torch.empty(B, dtype=torch.float32, device=pred.device)
        nobs = torch.empty(B, dtype=torch.float32, device=pred.device)
        part = torch.empty(int(L.rdq_l1_partial_bytes(B, n)), dtype=torch.uint8, device=pred.device)
        _hip.check(L.rdq_l1_forward(B, n, _hip.ptr(pred), _hip.ptr(y), _hip.ptr(mask), _hip.ptr(loss),
                                    _hip.ptr(nobs), _hip.ptr(part), _hip.stream_of(pred)), "rdq_l1_forward")
        if nobs_override is not None:          # shot-parallel: normalise by the global count
            loss = loss * (nobs / nobs_override)
            nobs = nobs_override.float().contiguous()
        ctx.save_for_backward(pred, y, mask, nobs)
        ctx.n = n
        return loss

    @staticmethod
    def backward(ctx, gout):
        pred, y, mask, nobs = ctx.saved_tensors
        B = pred.shape[0]
        dpred = torch.empty_like(pred)
        gout = gout.float().contiguous()
        _hip.check(_hip.lib().rdq_l1_backward(B, ctx.n, _hip.ptr(pred), _hip.ptr(y), _hip.ptr(mask),
                                              _hip.ptr(nobs), _hip.ptr(gout), _hip.ptr(dpred),
                                              _hip.stream_of(pred)), "rdq_l1_backward")
        return dpred, None, None, None


def l1_misfit(predicted, target, mask=None, nobs=None):
    return _L1Misfit.apply(predicted, target, mask, nobs)


class LossCalculator:
    """Observation + regularisation losses (losses.py:8-66)."""

    def __init__(self, regularization_method: RegularizationMethod):
        self.regularization_method = regularization_method
        self.global_nobs = None   # set by the engine when shots are sharded across ranks

    def observation_loss(self, predicted: torch.Tensor, target: torch.Tensor,
                         mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Per-model L1 misfit; with a mask, the mean over observed samples (losses.py:14-41)."""
        return l1_misfit(predicted, target, mask, self.global_nobs)

    def regularization_loss(self, mu: torch.Tensor, generator: Optional[torch.Generator] = None):
        return self.regularization_method.get_reg_loss(mu, generator=generator)

    def total_loss(self, obs_loss: torch.Tensor, reg_loss: torch.Tensor, reg_lambda: float) -> torch.Tensor:
        return obs_loss + reg_lambda * reg_loss
