"""LossCalculator (reference red_diffeq/core/losses.py:8-66) on the HIP L1 kernel (K5)."""
from typing import Optional

import torch

from .. import _hip
from .. import ops  # noqa: F401  (registers torch.ops.red_diffeq.*)
from ..regularization.base import RegularizationMethod


class _L1Misfit(torch.autograd.Function):
    """Per-model masked L1 misfit: forward torch.ops.red_diffeq.l1_misfit (K5), backward
    l1_misfit_backward (dpred = sign(pred - y) * mask * gout / nobs, exactly the autograd of
    losses.py:27-39).  nobs_override: the global observation count of a shot-sharded survey."""

    @staticmethod
    def forward(ctx, pred, y, mask, nobs_override):
        _hip.require_device(pred, y, mask)
        loss, nobs = torch.ops.red_diffeq.l1_misfit(pred, y, mask)
        if nobs_override is not None:          # shot-parallel: normalise by the global count
            loss = loss * (nobs / nobs_override)
            nobs = nobs_override.float().contiguous()
        ctx.save_for_backward(pred, y, mask, nobs)
        return loss

    @staticmethod
    def backward(ctx, gout):
        pred, y, mask, nobs = ctx.saved_tensors
        return torch.ops.red_diffeq.l1_misfit_backward(pred, y, mask, nobs, gout), None, None, None


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
