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
                io = dm.model.graph_io(x0.shape, x0.device) if t.dtype == torch.int64 and \
                    hasattr(dm.model, "graph_io") else None
                if io is not None:
                    # x_t and t written straight into the captured forward's static inputs
                    xs, ts = io
                    unet_ops.red_q_sample_into(dm, x0, t, noise, xs, ts)
                    eps_hat = dm.model.replay_static(xs, ts)
                    return unet_ops.red_epilogue(dm, xs, t, eps_hat, noise)
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
        """Models larger than image_size.  Height <= image_size - 2 (Marmousi 70x190): the reference's
        width-wise windows of size H with 0.5 blending in the overlaps (diffusion.py:85-155), same
        arithmetic order.  Taller models (configs[4], 500x3000; the reference has no path for them):
        2-D tiles of (image_size - 2)^2 placed by calculate_patches along both axes, blending weight
        = product of the two axes' 0.5-overlap weights.  All tiles go through ONE batched U-Net call;
        tiles are gathered and the gradient re-assembled by index (deterministic, no atomics)."""
        mu_c = diffusion_crop(mu)
        B, _, H, W = mu_c.shape
        if t is None:
            t = torch.randint(0, self._max_t(), (B,), generator=generator, device=mu.device, dtype=torch.long)
        if noise is None:
            noise = torch.randn(mu_c.shape, generator=generator, device=mu.device, dtype=mu.dtype)
        tp = tile_plan(H, W, self.input_size - 2, B, mu.device)
        x0 = diffusion_pad(tp.gather(mu_c.detach()))
        nz = diffusion_pad(tp.gather(noise))
        gp = diffusion_crop(self._eps_residual(x0, t.repeat(tp.P), nz))
        grad = tp.assemble(gp)
        reg = self._apply_time_weight(grad * mu_c, t)
        return reg.view(B, -1).mean(dim=1), grad.view(B, -1).mean(dim=1), t


def _axis_windows(n: int, m: int):
    """Windows of size m along an axis of length n and their blending weights: 1, and 0.5 where a
    window overlaps a neighbour (diffusion.py:135-141, including `w[-0:] = 0.5` when an overlap is
    empty: the reference then halves the whole window; the normalisation undoes it)."""
    pos, ov = calculate_patches(n, m)
    ws = []
    for i, (a, b) in enumerate(pos):
        w = torch.ones(b - a, dtype=torch.float32)
        if i > 0:
            w[:ov[i - 1]] = 0.5
        if i < len(pos) - 1:
            w[-ov[i]:] = 0.5
        ws.append(w)
    return pos, ws


class TilePlan:
    """Index maps of one (H, W, B) tiling: gather of the P tiles (patch-major batch p*B + b, the
    order of the reference's per-patch loop) and, per pixel, up to 4 covering tiles in tile order,
    so the blended sum accumulates in the reference's order without scatter-adds."""

    def __init__(self, H, W, m, B, device):
        if H <= m:                          # reference behaviour: width-wise windows of size H
            rows, rws = [(0, H)], [torch.ones(H)]
            cols, cws = _axis_windows(W, H)
        else:                               # 2-D tiles (new behaviour)
            rows, rws = _axis_windows(H, m)
            cols, cws = _axis_windows(W, m)
        mh, mw = rows[0][1] - rows[0][0], cols[0][1] - cols[0][0]
        self.P, self.B, self.mh, self.mw = len(rows) * len(cols), B, mh, mw
        self.rows, self.cols = rows, cols
        R = torch.tensor([[a + k for k in range(mh)] for a, _ in rows for _ in cols])
        C = torch.tensor([[a + k for k in range(mw)] for _ in rows for a, _ in cols])
        self.R, self.C = R.to(device), C.to(device)
        idx = torch.zeros(4, H, W, dtype=torch.int64)    # unused slots: index 0, weight 0
        wgt = torch.zeros(4, H, W, dtype=torch.float32)
        cnt = torch.zeros(H, W, dtype=torch.int64)
        p = 0
        for (r0, r1), wr in zip(rows, rws):
            for (c0, c1), wc in zip(cols, cws):
                ys, xs = torch.meshgrid(torch.arange(r0, r1), torch.arange(c0, c1), indexing="ij")
                q = cnt[r0:r1, c0:c1]
                idx[q, ys, xs] = p * B * mh * mw + (ys - r0) * mw + (xs - c0)
                wgt[q, ys, xs] = wr[:, None] * wc[None, :]
                cnt[r0:r1, c0:c1] += 1
                p += 1
        if int(cnt.max()) > 4 or int(cnt.min()) < 1:
            raise ValueError(f"tiling of {H}x{W} by {m}: coverage {int(cnt.min())}..{int(cnt.max())}")
        boff = (torch.arange(B, dtype=torch.int64) * mh * mw).view(1, B, 1, 1)
        self.idx = (idx.view(4, 1, H, W) + boff).to(device)          # (4, B, H, W)
        self.wgt = wgt.to(device)
        wsum = torch.zeros(H, W)
        for q in range(4):                                           # reference order: 0 + w0 + w1 ...
            wsum = wsum + wgt[q]
        self.wsum = wsum.clamp(min=1e-8).to(device)

    def gather(self, x):
        """(B,1,H,W) -> (P*B, 1, mh, mw), patch-major."""
        t = x[:, 0][:, self.R[:, :, None], self.C[:, None, :]]       # (B, P, mh, mw)
        return t.transpose(0, 1).reshape(self.P * self.B, 1, self.mh, self.mw)

    def assemble(self, gp):
        """Blend per-tile fields (P*B, 1, mh, mw) back to (B, 1, H, W)."""
        flat = gp.reshape(-1)
        acc = torch.zeros(self.idx.shape[1:], dtype=gp.dtype, device=gp.device)
        for q in range(4):
            acc = acc + flat[self.idx[q]] * self.wgt[q]
        return (acc / self.wsum).unsqueeze(1)


_TILE_PLANS = {}


def tile_plan(H, W, m, B, device):
    key = (H, W, m, B, str(device))
    if key not in _TILE_PLANS:
        _TILE_PLANS[key] = TilePlan(H, W, m, B, device)
    return _TILE_PLANS[key]


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
