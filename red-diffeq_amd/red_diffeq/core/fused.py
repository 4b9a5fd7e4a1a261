"""The inversion loop's serial tail on the HIP kernels of csrc/loop.hip (C ABI
include/red_diffeq_loop.h): fused Adam + clamp (K11) and fused MAE/RMSE/SSIM (K12).

Reference behaviour: red_diffeq/core/inversion.py:80-111 (torch.optim.Adam, clamp_(-1, 1),
CosineAnnealingLR, MetricsCalculator).  The learning-rate schedule is torch's recursive
CosineAnnealingLR formula evaluated on the host (a scalar per iteration, no device sync)."""
import math

import torch

from .. import _hip
from .. import ops  # noqa: F401  (registers torch.ops.red_diffeq.*)


class CosineLR:
    """torch.optim.lr_scheduler.CosineAnnealingLR(T_max, eta_min), recursive form, for one group."""

    def __init__(self, base_lr, T_max, eta_min=0.0):
        self.base_lr, self.T_max, self.eta_min = float(base_lr), T_max, float(eta_min)
        self.lr = self.base_lr
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        e, T, b, m = self.last_epoch, self.T_max, self.base_lr, self.eta_min
        if (e - 1 - T) % (2 * T) == 0:
            self.lr = self.lr + (b - m) * (1 - math.cos(math.pi / T)) / 2
        else:
            self.lr = (1 + math.cos(math.pi * e / T)) / (1 + math.cos(math.pi * (e - 1) / T)) * (self.lr - m) + m
        return self.lr


class FusedAdamClamp:
    """torch.optim.Adam([param], lr, betas, eps) step + param.clamp_(lo, hi), one HIP launch."""

    def __init__(self, param, lr, betas=(0.9, 0.999), eps=1e-8, clamp=(-1.0, 1.0)):
        _hip.require_device(param)
        if not param.is_contiguous():
            raise ValueError("FusedAdamClamp needs a contiguous parameter")
        self.param = param
        self.lr = float(lr)
        self.beta1, self.beta2 = float(betas[0]), float(betas[1])
        self.eps = float(eps)
        self.clamp = clamp
        self.exp_avg = torch.zeros_like(param)
        self.exp_avg_sq = torch.zeros_like(param)
        self.t = 0

    def zero_grad(self):
        self.param.grad = None

    @torch.no_grad()
    def step(self, lr=None, guard=None):
        """guard: optional device int32 word; when it is non-zero at execution time the step is a
        no-op on the device (rdq_adam_step), e.g. the FWI status word of a failed persistent launch."""
        if lr is not None:
            self.lr = float(lr)
        g = self.param.grad
        if g is None:
            return
        g = g.contiguous()
        self.t += 1
        bc1 = 1 - self.beta1 ** self.t                  # torch/optim/adam.py (_multi_tensor_adam)
        bc2 = 1 - self.beta2 ** self.t
        step_size = (self.lr / bc1) * -1
        lo, hi = self.clamp if self.clamp is not None else (0.0, 0.0)
        torch.ops.red_diffeq.adam_clamp_(self.param.data, g, self.exp_avg, self.exp_avg_sq, self.beta1, self.beta2,
                                         self.eps, step_size, bc2 ** 0.5, self.clamp is not None, float(lo),
                                         float(hi), guard)


def metrics(pred, true_norm):
    """(mae, rmse, ssim) per model, (3, B) float32 on the device, no host sync
    (torch.ops.red_diffeq.metrics, K12)."""
    _hip.require_device(pred)
    return torch.ops.red_diffeq.metrics(pred, true_norm)
