"""MetricsCalculator (reference red_diffeq/core/metrics.py:7-46): MAE, RMSE, SSIM per model in
normalised units, on the device, off the gradient path."""
from typing import Tuple

import torch

from ..utils.data_trans import v_normalize
from ..utils.ssim import SSIM


class MetricsCalculator:

    def __init__(self, ssim_loss: SSIM):
        self.ssim_loss = ssim_loss

    @torch.no_grad()
    def calculate(self, mu: torch.Tensor, mu_true: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        B = mu.shape[0]
        pred = mu.detach()
        true = v_normalize(mu_true).to(mu.device)
        mae = torch.mean(torch.abs(pred - true), dim=(1, 2, 3))
        rmse = torch.sqrt(torch.mean((pred - true) ** 2, dim=(1, 2, 3)))
        p01, t01 = (pred + 1) / 2, (true + 1) / 2
        ssim = torch.zeros(B, device=mu.device)
        for i in range(B):
            ssim[i] = self.ssim_loss(p01[i:i + 1], t01[i:i + 1])
        return mae, rmse, ssim
