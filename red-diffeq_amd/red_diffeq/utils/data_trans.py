"""Data transforms (reference red_diffeq/utils/data_trans.py:8-153).

Host-side helpers called once per ``InversionEngine.optimize`` (noise, missing traces, initial
model); the per-iteration denormalisation is fused into the HIP coefficient kernel.
"""
from typing import Optional

import numpy as np
import torch
from scipy.ndimage import gaussian_filter


def v_normalize(v):
    """Velocity [1500, 4500] m/s -> [-1, 1] (data_trans.py:8-10)."""
    return (v - 1500) / 3000 * 2 - 1


def v_denormalize(v_norm):
    """[-1, 1] -> velocity (data_trans.py:13-15); FWIForward fuses exactly this map."""
    return (v_norm + 1) / 2 * 3000 + 1500


def s_normalize_none(s):
    return s


def s_normalize(s):
    return (s + 20) / 80 * 2 - 1


def s_denormalize(s_norm):
    return (s_norm + 1) / 2 * 80 - 20


def add_noise_to_seismic(y: torch.Tensor, std: float, noise_type: str = "gaussian",
                         generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Gaussian or Laplace noise (data_trans.py:33-62), same RNG draw order."""
    assert std >= 0, "The standard deviation/scale of the noise must be greater than 0"
    assert noise_type in ["gaussian", "laplace"], f"Unknown noise type: {noise_type}"
    if std == 0:
        return y
    if noise_type == "gaussian":
        noise = torch.randn(y.shape, generator=generator, device=y.device, dtype=y.dtype) * std
    else:
        u = torch.rand(y.shape, generator=generator, device=y.device, dtype=y.dtype) - 0.5
        noise = -std * torch.sign(u) * torch.log(1 - 2 * torch.abs(u))
    return y + noise


def prepare_initial_model(v_true: torch.Tensor, initial_type: str = None, sigma: float = None,
                          linear_coeff: float = 1.0) -> torch.Tensor:
    """Initial model (data_trans.py:65-107): scipy-smoothed, homogeneous or linear, normalised."""
    assert initial_type in ["smoothed", "homogeneous", "linear"], \
        "please choose from 'smoothed', 'homogeneous', and 'linear'"
    device = v_true.device
    v_np = v_normalize(v_true.clone().cpu().numpy())
    if initial_type == "smoothed":
        v_blurred = gaussian_filter(v_np, sigma=sigma)
    elif initial_type == "homogeneous":
        v_blurred = np.full_like(v_np, np.min(v_np[0, 0, 0, :]))
    else:
        v_min, v_max = np.min(v_np), np.max(v_np)
        height = v_np.shape[2]
        grad = np.linspace(v_min, v_max, height).reshape(-1, 1)
        v_blurred = np.tile(grad, (1, v_np.shape[3])).reshape(1, 1, height, -1)
    return torch.tensor(v_blurred, dtype=torch.float32, device=device)


def missing_trace(y: torch.Tensor, num_missing: int, return_mask: bool = True,
                  generator: Optional[torch.Generator] = None):
    """Zero the same random receivers for every shot of a model (data_trans.py:110-153)."""
    assert num_missing >= 0, "The number of missing traces must be >= 0"
    batch_size, _, _, num_traces = y.shape
    mask = torch.ones_like(y, device=y.device)
    if num_missing == 0:
        return (y, mask) if return_mask else y
    y_missing = y.clone()
    for b in range(batch_size):
        idx = torch.randperm(num_traces, generator=generator, device=y.device)[:num_missing]
        y_missing[b, :, :, idx] = 0
        mask[b, :, :, idx] = 0
    return (y_missing, mask) if return_mask else y_missing
