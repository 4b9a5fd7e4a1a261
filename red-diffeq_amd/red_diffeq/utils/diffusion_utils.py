"""Diffusion helpers (reference red_diffeq/utils/diffusion_utils.py:4-14)."""
import torch
import torch.nn.functional as F


def extract(a, t, x_shape):
    """Gather a[t] and reshape to broadcast over x_shape (diffusion_utils.py:4-7)."""
    b = t.shape[0]
    out = a.gather(-1, t)
    return out.reshape(b, *((1,) * (len(x_shape) - 1)))


def diffusion_pad(x: torch.Tensor) -> torch.Tensor:
    """Zero-pad by one pixel on every side (70x70 -> 72x72), diffusion_utils.py:9-11."""
    return F.pad(x, (1, 1, 1, 1), mode="constant", value=0)


def diffusion_crop(x: torch.Tensor) -> torch.Tensor:
    """Inverse of diffusion_pad, diffusion_utils.py:13-14."""
    return x[:, :, 1:-1, 1:-1]
