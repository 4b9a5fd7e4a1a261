"""DiffusionFWI (reference diffusion_bench/diffusionfwi.py:79-366): reverse diffusion over
`diffusion_ts` steps; at each step denoise the current model with p_mean_variance
(diffusionfwi.py:97-178), then, except at t = 0, run `ts` Adam iterations of FWI on the denoised
model with the gradient tricks of diffusionfwi.py:259-317 (normalise by the first iteration's
max |g|, optional Gaussian smoothing, norm clipping, optional 3x3 blur, clamp to [-1, 1]).

Same constructor, same optimize() signature, same returned (mu, per-model histories).  On the
MI355X path: the forward / adjoint are the HIP kernels behind FWIForward, the denoiser is the HIP
U-Net, the masked L1 misfit is the HIP kernel of LossCalculator, Adam (+ clamp) is the fused HIP
step (fresh moments every diffusion step, as the reference re-creates torch.optim.Adam), metrics
are the fused HIP kernel with histories kept on the device.  Patch denoising batches every patch
through ONE U-Net call (the reference loops over patches).
"""
import math

import torch
import torch.nn.functional as F
from tqdm.auto import tqdm

from red_diffeq.core.fused import FusedAdamClamp, metrics as fused_metrics
from red_diffeq.core.inversion import k12_covers
from red_diffeq.core.losses import LossCalculator
from red_diffeq.core.metrics import MetricsCalculator
from red_diffeq.utils.data_trans import add_noise_to_seismic, missing_trace, v_normalize
from red_diffeq.utils.diffusion_utils import diffusion_crop, diffusion_pad


def split_data_to_patches(data, kernel_size, stride):
    """(B,C,H,W) -> (B*nh*nw, C, kh, kw), patches in (b, i, j) order (diffusionfwi.py:32-43)."""
    B, C, H, W = data.shape
    ph, pw = kernel_size
    sh, sw = stride
    p = data.unfold(2, ph, sh).unfold(3, pw, sw)
    return p.permute(0, 2, 3, 1, 4, 5).reshape(-1, C, ph, pw)


def merge_patches_to_data(patches, output_size, kernel_size, stride, batch=1):
    """Overlap-average of split_data_to_patches' output (diffusionfwi.py:46-76), per model, as one
    fold of the patch sums divided by a fold of the counts."""
    N, C, ph, pw = patches.shape
    H, W = output_size
    nh = (H - ph) // stride[0] + 1
    nw = (W - pw) // stride[1] + 1
    cols = patches.reshape(batch, nh * nw, C * ph * pw).transpose(1, 2)
    merged = F.fold(cols, (H, W), (ph, pw), stride=stride)
    count = F.fold(torch.ones_like(cols[:1]), (H, W), (ph, pw), stride=stride)
    return merged / count.clamp(min=1)


def _gaussian_smooth(g, sigma):
    """scipy.ndimage.gaussian_filter(g, sigma=[0, 0, s, s]) on the device: separable kernel of
    radius int(4 s + 0.5), 'reflect' (half-sample symmetric) boundaries (diffusionfwi.py:289-295)."""
    r = int(4.0 * sigma + 0.5)
    x = torch.arange(-r, r + 1, dtype=torch.float64)
    k = torch.exp(-0.5 * (x / sigma) ** 2)
    k = (k / k.sum()).to(g.device, torch.float32)
    B, C, H, W = g.shape

    def refl(n):   # index map of half-sample-symmetric padding by r
        i = torch.arange(-r, n + r, device=g.device)
        p = 2 * n
        i = torch.remainder(i, p)
        return torch.where(i >= n, p - 1 - i, i)

    y = g[..., refl(H), :]
    y = F.conv2d(y.reshape(B * C, 1, H + 2 * r, W), k.view(1, 1, -1, 1)).reshape(B, C, H, W)
    y = y[..., refl(W)]
    return F.conv2d(y.reshape(B * C, 1, H, W + 2 * r), k.view(1, 1, 1, -1)).reshape(B, C, H, W)


def _blur3(x, sigma=0.4):
    """torchvision gaussian_blur(kernel [3, 3], sigma [0.4, 0.4]): separable, reflect padding
    (diffusionfwi.py:311-316)."""
    t = torch.linspace(-1.0, 1.0, 3, device=x.device)
    k = torch.exp(-0.5 * (t / sigma) ** 2)
    k = k / k.sum()
    B, C, H, W = x.shape
    y = F.pad(x.reshape(B * C, 1, H, W), (1, 1, 1, 1), mode="reflect")
    y = F.conv2d(y, k.view(1, 1, 3, 1))
    y = F.conv2d(y, k.view(1, 1, 1, 3))
    return y.reshape(B, C, H, W)


class DiffusionFWI:

    def __init__(self, diffusion_model, fwi_forward, ssim_loss):
        self.diffusion_model = diffusion_model
        self.fwi_forward = fwi_forward
        self.ssim_loss = ssim_loss
        self.device = diffusion_model.device

    def _condition(self, denoised, current, step):
        """Hook after denoising (ILVR_FWI adds its low-frequency conditioning here)."""
        return denoised

    @torch.no_grad()
    def _apply_diffusion_denoising_with_patches(self, current_model, diffusion_step, kernel_size=None,
                                                stride=None, use_patches=False):
        """img_mean of one reverse step (diffusionfwi.py:97-178)."""
        dm = self.diffusion_model
        B, _, H, W = current_model.shape
        kernel_size = kernel_size or [H, H]
        stride = stride or [1, 1]
        image_size = dm.image_size[0] if isinstance(dm.image_size, (tuple, list)) else dm.image_size
        unpadded = image_size - 2
        if not (use_patches and (W != H or W > image_size)):
            t = torch.full((B,), diffusion_step, device=current_model.device, dtype=torch.long)
            mean, _, _, _ = dm.p_mean_variance(x=diffusion_pad(current_model), t=t, x_self_cond=None,
                                               clip_denoised=True)
            return diffusion_crop(mean).clamp(-1.0, 1.0)
        patches = split_data_to_patches(current_model, kernel_size, stride)
        P = patches.shape[0]
        x = F.interpolate(patches, size=(unpadded, unpadded), mode="bilinear", align_corners=False)
        t = torch.full((P,), diffusion_step, device=current_model.device, dtype=torch.long)
        mean, _, _, _ = dm.p_mean_variance(x=diffusion_pad(x), t=t, x_self_cond=None, clip_denoised=True)
        den = diffusion_crop(mean).clamp(-1.0, 1.0)
        den = F.interpolate(den, size=tuple(kernel_size), mode="bilinear", align_corners=False)
        return merge_patches_to_data(den, [H, W], kernel_size, stride, batch=B)

    def optimize(self, mu, mu_true, y, fwi_forward, ts=300, diffusion_ts=500, lr=0.03, noise_std=0.0,
                 noise_type="gaussian", missing_number=0, grad_norm=True, grad_smooth=None, model_blur=False,
                 grad_clip=1.0, use_patches=False, patch_kernel_size=None, patch_stride=None):
        if mu.shape[0] != y.shape[0]:
            raise ValueError("Batch size mismatch between velocity and seismic data")
        if fwi_forward is None or not callable(fwi_forward):
            raise ValueError("fwi_forward must be a callable forward modeling function")
        fwi_forward = fwi_forward.to(self.device)
        B = mu.shape[0]
        mu = mu.float().clone().detach().to(self.device)
        true_norm = v_normalize(mu_true.float().to(self.device)).contiguous()
        y = add_noise_to_seismic(y, noise_std, noise_type=noise_type)
        y, mask = missing_trace(y, missing_number, return_mask=True)
        y = y.to(self.device)
        mask = mask.to(self.device) if missing_number else None
        loss_calc = LossCalculator(None)
        # K12 when ssim_loss is the reference's SSIM, else the module itself (reference MetricsCalculator)
        metrics_calc = None if k12_covers(self.ssim_loss) else MetricsCalculator(self.ssim_loss)
        keys = ("total_losses", "obs_losses", "ssim", "mae", "rmse")
        hist = torch.zeros(diffusion_ts, len(keys), B, dtype=torch.float32, device=self.device)

        current = mu
        for row, step in enumerate(tqdm(range(diffusion_ts - 1, -1, -1), desc="DiffusionFWI", unit="step",
                                        position=0)):
            denoised = self._apply_diffusion_denoising_with_patches(current, step, kernel_size=patch_kernel_size,
                                                                    stride=patch_stride, use_patches=use_patches)
            denoised = self._condition(denoised, current, step)
            if step != 0:
                mu_opt = denoised.clone().detach().contiguous().requires_grad_(True)
                opt = FusedAdamClamp(mu_opt, lr=lr, clamp=None if model_blur else (-1.0, 1.0))
                grad_max = None
                for it in range(ts):
                    opt.zero_grad()
                    loss_obs = loss_calc.observation_loss(fwi_forward(mu_opt), y, mask=mask)
                    loss_obs.sum().backward()
                    with torch.no_grad():
                        g = mu_opt.grad
                        if grad_norm:
                            if it == 0:
                                grad_max = torch.max(torch.abs(g)).item()
                            if grad_max is not None and grad_max > 0:
                                g /= grad_max
                        if grad_smooth is not None and grad_smooth > 0:
                            mu_opt.grad = _gaussian_smooth(g, grad_smooth)
                            grad_max = torch.max(torch.abs(mu_opt.grad)).item()
                        if grad_clip is not None and grad_clip > 0 and grad_max is not None and grad_max > 0:
                            torch.nn.utils.clip_grad_norm_([mu_opt], grad_clip * grad_max)
                    # a gradient from a failed persistent FWI launch is never applied (device guard)
                    opt.step(guard=getattr(fwi_forward, "status_word", lambda: None)())
                    if model_blur:
                        with torch.no_grad():
                            mu_opt.data = _blur3(mu_opt.data).clamp_(-1.0, 1.0).contiguous()
                            opt.param = mu_opt
                current = mu_opt.detach()
                check = getattr(fwi_forward, "check", None)
                if callable(check):
                    check()      # one sync per reverse step: raise before the next step builds on it
            else:
                current = denoised.detach()
            with torch.no_grad():
                obs = loss_calc.observation_loss(fwi_forward(current), y, mask=mask)
                if metrics_calc is None:
                    m = fused_metrics(current, true_norm)                 # (mae, rmse, ssim)
                else:                                                     # the caller's own SSIM module
                    m = metrics_calc.calculate(current, mu_true.float().to(self.device))
                hist[row, 0] = obs
                hist[row, 1] = obs
                hist[row, 2] = m[2]
                hist[row, 3] = m[0]
                hist[row, 4] = m[1]
        H = hist.cpu().numpy()
        results = [{k: [H[s, j, i] for s in range(diffusion_ts)] for j, k in enumerate(keys)} for i in range(B)]
        return current, results


del math
