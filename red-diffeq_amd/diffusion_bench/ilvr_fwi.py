"""ILVR_FWI (reference diffusion_bench/ilvr_fwi.py:41-326): DiffusionFWI with ILVR conditioning
after each denoising step (t > 0),

    denoised' = clamp(denoised - a LF(denoised) + a LF(q_sample(current, t, eps)), -1, 1),

LF = downsample by 1/N then upsample by N with the antialiased bicubic resampler of
diffusion_bench/resizer.py (N from the 'linear' (16 -> 2) or 'stepwise' ([32, 16, 8, 4]) schedule,
indexed by t).  The resampler is restated here as dense per-axis weight matrices applied with two
small matmuls on the device (same kernel, same coordinate mapping, same mirror boundary, same
per-output normalisation as resizer.py:63-83); sizes that do not round-trip are brought back with
bilinear interpolation as the reference does (ilvr_fwi.py:303-316).
"""
import numpy as np
import torch
import torch.nn.functional as F

from .diffusionfwi import DiffusionFWI


def _cubic(x):
    ax = np.abs(x)
    return ((1.5 * ax ** 3 - 2.5 * ax ** 2 + 1) * (ax <= 1)
            + (-0.5 * ax ** 3 + 2.5 * ax ** 2 - 4 * ax + 2) * ((ax > 1) & (ax <= 2)))


def resize_matrix(in_len, out_len, scale):
    """(out_len, in_len) weights of the bicubic resampler along one axis, antialiased when scale < 1."""
    aa = scale < 1
    width = 4.0 / scale if aa else 4.0
    kern = (lambda u: scale * _cubic(scale * u)) if aa else _cubic
    o = np.arange(1, out_len + 1, dtype=np.float64)
    centre = (o - (out_len - in_len * scale) / 2) / scale + 0.5 * (1 - 1 / scale)
    left = np.floor(centre - width / 2)
    taps = int(np.ceil(width)) + 2
    idx = left[:, None] + np.arange(taps)[None, :] - 1                 # (out, taps), 0-based source
    w = kern(centre[:, None] - idx - 1)
    s = w.sum(axis=1)
    s[s == 0] = 1.0
    w = w / s[:, None]
    period = 2 * in_len                                                 # mirror: 0..n-1, n-1..0
    m = np.mod(idx.astype(np.int64), period)
    src = np.where(m < in_len, m, period - 1 - m)
    M = np.zeros((out_len, in_len))
    np.add.at(M, (np.repeat(np.arange(out_len), taps), src.ravel()), w.ravel())
    return M


def resize(x, scale, in_hw=None):
    """Resize the last two axes of x by `scale` (output ceil(in * scale)); in_hw: the input size the
    resampler is built for (rows / columns beyond it are ignored, as the reference's index gather
    does when the declared shape is smaller than the tensor)."""
    H, W = in_hw or x.shape[-2:]
    oh, ow = int(np.ceil(H * scale)), int(np.ceil(W * scale))
    Mh = torch.from_numpy(resize_matrix(H, oh, scale)).to(x.device, torch.float32)
    Mw = torch.from_numpy(resize_matrix(W, ow, scale)).to(x.device, torch.float32)
    y = torch.matmul(Mh, x[..., :H, :W])                    # rows first (resizer.py: sorted dims)
    return torch.matmul(y, Mw.t())


class ILVR_FWI(DiffusionFWI):

    def __init__(self, diffusion_model, fwi_forward, ssim_loss):
        super().__init__(diffusion_model, fwi_forward, ssim_loss)
        self.randn_like = torch.randn_like            # the q_sample noise draw (injectable for tests)

    def optimize(self, mu, mu_true, y, fwi_forward, ts=300, diffusion_ts=500, lr=0.03, noise_std=0.0,
                 noise_type="gaussian", missing_number=0, grad_norm=True, grad_smooth=None, model_blur=False,
                 grad_clip=1.0, use_ilvr=True, ilvr_weight=0.05, ilvr_down_schedule="linear", use_patches=False,
                 patch_kernel_size=None, patch_stride=None):
        self.use_ilvr = use_ilvr
        self.ilvr_weight = ilvr_weight
        if ilvr_down_schedule == "linear":
            self.down_n = np.linspace(16, 2, diffusion_ts).astype(int)
        elif ilvr_down_schedule == "stepwise":
            ns = [32, 16, 8, 4]
            self.down_n = np.repeat(ns, diffusion_ts // len(ns))
            if len(self.down_n) < diffusion_ts:
                self.down_n = np.pad(self.down_n, (0, diffusion_ts - len(self.down_n)), constant_values=ns[-1])
        else:
            raise ValueError(f"Unknown ilvr_down_schedule: {ilvr_down_schedule}")
        return super().optimize(mu, mu_true, y, fwi_forward, ts=ts, diffusion_ts=diffusion_ts, lr=lr,
                                noise_std=noise_std, noise_type=noise_type, missing_number=missing_number,
                                grad_norm=grad_norm, grad_smooth=grad_smooth, model_blur=model_blur,
                                grad_clip=grad_clip, use_patches=use_patches, patch_kernel_size=patch_kernel_size,
                                patch_stride=patch_stride)

    def _condition(self, denoised, current, step):
        if not self.use_ilvr or step <= 0:
            return denoised
        return self._apply_ilvr(denoised, current, step)

    @torch.no_grad()
    def _apply_ilvr(self, denoised, current_model, t):
        n = int(self.down_n[t])
        H, W = denoised.shape[2], denoised.shape[3]
        noised = self.diffusion_model.q_sample(current_model, torch.tensor([t], device=denoised.device),
                                               self.randn_like(current_model))

        def lowpass(x):
            d = resize(x, 1.0 / n)
            u = resize(d, float(n), in_hw=(int(H / n), int(W / n)))
            if u.shape[2:] != (H, W):
                u = F.interpolate(u, size=(H, W), mode="bilinear", align_corners=False)
            return u

        out = denoised - self.ilvr_weight * lowpass(denoised) + self.ilvr_weight * lowpass(noised)
        return out.clamp(-1.0, 1.0)
