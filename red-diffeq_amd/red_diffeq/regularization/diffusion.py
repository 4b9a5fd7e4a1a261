"""RED-DiffEq regulariser (reference red_diffeq/regularization/diffusion.py:7-200).

loss = mean((eps_hat' - eps).detach() * mu) [* sqrt((1-abar)/abar) if use_time_weight], so
d loss / d mu = (eps_hat' - eps) / (H*W): the U-Net runs forward only.  RNG draw order per call
is the reference's: t = randint(0, T) first, then eps = randn(mu.shape).
"""
import math
from typing import List, Optional, Tuple

import torch

from ..utils.diffusion_utils import diffusion_crop, diffusion_pad, extract


def calculate_patches(width: int, height: int) -> Tuple[List[Tuple[int, int]], List[int]]:
    """Width-wise windows of size `height` with even spacing (diffusion.py:7-27)."""
    m, n = height, width
    k = math.ceil(n / m)
    if k == 1:
        return [(0, n)], []
    s = (n - m) / (k - 1)
    pos = [(n - m, n) if i == k - 1 else (int(i * s), min(int(i * s) + m, n)) for i in range(k)]
    return pos, [pos[i][1] - pos[i + 1][0] for i in range(k - 1)]


class RED_DiffEq:

    def __init__(self, diffusion_model, use_time_weight: bool = False, sigma_x0: float = 0.0001,
                 fixed_timestep: int = None):
        self.diffusion_model = diffusion_model
        self.use_time_weight = use_time_weight
        self.sigma_x0 = sigma_x0
        self.fixed_timestep = fixed_timestep
        image_size = getattr(diffusion_model, "image_size", 72)
        self.input_size = image_size[0] if isinstance(image_size, (tuple, list)) else image_size

    def _apply_time_weight(self, tensor, t):
        if not self.use_time_weight:
            return tensor
        g = extract(self.diffusion_model.alphas_cumprod, t, tensor.shape)
        return tensor * torch.sqrt((1.0 - g) / g)

    def _max_t(self):
        return self.fixed_timestep if self.fixed_timestep is not None else self.diffusion_model.num_timesteps

    def _eps_residual(self, x0, t, noise):
        """(eps_hat' - eps) for padded 72x72 inputs: q_sample -> U-Net -> clip/re-derive.
        For the pred_noise objective (the RED-DiffEq configs) the prologue / epilogue are the
        fused HIP kernels; other objectives use GaussianDiffusion.model_predictions."""
        dm = self.diffusion_model
        with torch.no_grad():
            if getattr(dm, "objective", None) == "pred_noise" and x0.is_cuda and not dm.self_condition:
                from ..models import unet_ops
                x_t = unet_ops.red_q_sample(dm, x0, t, noise)
                eps_hat = dm.model(x_t, t, None)
                return unet_ops.red_epilogue(dm, x_t, t, eps_hat, noise)
            x_t = dm.q_sample(x0, t=t, noise=noise)
            pred = dm.model_predictions(x_t, t=t, x_self_cond=None, clip_x_start=True,
                                        rederive_pred_noise=True)
            return (pred.pred_noise - noise).detach()

    def get_reg_loss(self, mu, generator: Optional[torch.Generator] = None, t=None, noise=None):
        """-> (reg per model (B,), mean residual per model (B,), t (B,)).  ``t``/``noise`` may be
        injected (parity tests: GPU and CPU RNG streams differ)."""
        B = mu.shape[0]
        if t is None:
            t = torch.randint(0, self._max_t(), (B,), generator=generator, device=mu.device, dtype=torch.long)
        if noise is None:
            noise = torch.randn(mu.shape, generator=generator, device=mu.device, dtype=mu.dtype)
        g = self._eps_residual(mu.detach(), t, noise)
        reg = self._apply_time_weight(g * mu, t)
        return reg.view(B, -1).mean(dim=1), g.view(B, -1).mean(dim=1), t

    def get_reg_loss_patched(self, mu, generator: Optional[torch.Generator] = None, t=None, noise=None):
        """Width > image_size (Marmousi 70x190): overlapping 70-wide windows, 0.5 blending
        (diffusion.py:85-155).  All windows go through ONE batched U-Net call."""
        mu_c = diffusion_crop(mu)
        B, _, H, W = mu_c.shape
        pos, ov = calculate_patches(W, H)
        if t is None:
            t = torch.randint(0, self._max_t(), (B,), generator=generator, device=mu.device, dtype=torch.long)
        if noise is None:
            noise = torch.randn(mu_c.shape, generator=generator, device=mu.device, dtype=mu.dtype)
        P = len(pos)
        x0 = torch.cat([diffusion_pad(mu_c[:, :, :, a:b].detach()) for a, b in pos], dim=0)
        nz = torch.cat([diffusion_pad(noise[:, :, :, a:b]) for a, b in pos], dim=0)
        gp = diffusion_crop(self._eps_residual(x0, t.repeat(P), nz))
        grad = torch.zeros_like(mu_c)
        wmap = torch.zeros_like(mu_c)
        for i, (a, b) in enumerate(pos):
            w = torch.ones(b - a, device=mu.device)
            if i > 0:
                w[:ov[i - 1]] = 0.5
            if i < P - 1:
                w[-ov[i]:] = 0.5
            w = w.view(1, 1, 1, -1)
            grad[:, :, :, a:b] += gp[i * B:(i + 1) * B] * w
            wmap[:, :, :, a:b] += w
        grad = grad / wmap.clamp(min=1e-8)
        reg = self._apply_time_weight(grad * mu_c, t)
        return reg.view(B, -1).mean(dim=1), grad.view(B, -1).mean(dim=1), t


class RED_DiffEq_POST_PROCESS:
    """Deterministic denoising post-process (diffusion.py:158-200)."""

    def __init__(self, diffusion_model):
        self.diffusion_model = diffusion_model

    def generate_time_tensor(self, timesteps, mu):
        return torch.full((mu.shape[0],), timesteps, device=mu.device, dtype=torch.long)

    def generate_noisy_sample(self, mu, time_tensor):
        noise = torch.randn_like(mu)
        x_t_norm = self.diffusion_model.q_sample(self.diffusion_model.normalize(mu), t=time_tensor, noise=noise)
        return self.diffusion_model.unnormalize(x_t_norm), noise, mu

    @torch.no_grad()
    def diffusion_denoise(self, mu, timesteps):
        dm = self.diffusion_model
        if timesteps > dm.num_timesteps:
            raise ValueError(f"timesteps ({timesteps}) exceeds model's num_timesteps ({dm.num_timesteps})")
        mu01 = (mu + 1) / 2
        x_t, _, _ = self.generate_noisy_sample(mu01, self.generate_time_tensor(timesteps, mu01))
        x_start = None
        for t in reversed(range(timesteps)):
            sc = x_start if dm.self_condition else None
            x_t_norm, xs_norm = dm.p_sample_deterministic(dm.normalize(x_t), t=t, x_self_cond=sc)
            x_t = dm.unnormalize(x_t_norm)
            x_start = dm.unnormalize(xs_norm) if xs_norm is not None else None
        return x_t
