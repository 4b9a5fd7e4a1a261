"""InversionEngine (reference red_diffeq/core/inversion.py:12-129), same API and loop order.

Per iteration: [diffusion: eps_x0 ~ N(0,1); x0 = mu + sigma_x0 eps_x0] -> seis = fwi_forward(
x0[:, :, 1:-1, 1:-1]) -> L1 misfit -> regulariser -> backward (HIP adjoint) -> Adam -> clamp to
[-1,1] -> cosine LR step -> metrics.  RNG draw order matches the reference
(eps_x0, then the regulariser's t, then eps).

Shot-parallel inversion: when ``fwi_forward.shots`` covers a subset of the sources
and a torch.distributed process group is initialised, each rank models its shots only; the
misfit is normalised by the global observation count; the data-term gradient is summed over
ranks by ONE all-reduce inside backward (``_GradAllReduce``); the regulariser, Adam and the
metrics run replicated (identical seeds -> identical draws on every rank).
"""
from typing import Optional

import torch
import torch.distributed as dist
from tqdm.auto import tqdm

from ..regularization.base import RegularizationMethod
from ..utils.data_trans import add_noise_to_seismic, missing_trace
from ..utils.data_trans import v_normalize
from ..utils.ssim import SSIM
from .fused import CosineLR, FusedAdamClamp, metrics as fused_metrics
from .losses import LossCalculator


class _GradAllReduce(torch.autograd.Function):
    """Identity forward; backward sums the incoming gradient over the process group."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=ctx.group)
        return g, None


def grad_all_reduce(x, group=None):
    return _GradAllReduce.apply(x, group)


def shot_slice(fwi_forward, ns_total):
    """(start, stop) of the shots the operator models, or None when it models them all."""
    shots = getattr(fwi_forward, "shots", None)
    if shots is None or (shots[0] == 0 and shots[1] == ns_total):
        return None
    return shots


class InversionEngine:

    def __init__(self, diffusion_model, ssim_loss: SSIM, regularization: Optional[str] = None,
                 use_time_weight: bool = False, sigma_x0: float = 0.0001, fixed_timestep: int = None,
                 show_progress: bool = True):
        self.diffusion_model = diffusion_model
        self.ssim_loss = ssim_loss
        self.device = diffusion_model.device
        self.sigma_x0 = sigma_x0
        self.show_progress = show_progress
        self.regularization_method = RegularizationMethod(
            regularization, diffusion_model, use_time_weight=use_time_weight, sigma_x0=sigma_x0,
            fixed_timestep=fixed_timestep)

    def optimize(self, mu: torch.Tensor, mu_true: torch.Tensor, y: torch.Tensor, fwi_forward, ts: int = 300,
                 lr: float = 0.03, reg_lambda: float = 0.01, noise_std: float = 0.0, noise_type: str = "gaussian",
                 missing_number: int = 0, regularization: Optional[str] = None, process_group=None):
        if mu.shape[0] != y.shape[0]:
            raise ValueError("Batch size mismatch between velocity and seismic data")
        if regularization not in ["diffusion", "l2", "tv", "hybrid", None]:
            raise ValueError(f"Unknown regularization: {regularization}")
        if fwi_forward is None or not callable(fwi_forward):
            raise ValueError("fwi_forward must be a callable forward modeling function")
        fwi_forward = fwi_forward.to(self.device)
        if regularization is not None:
            rm = self.regularization_method
            self.regularization_method = RegularizationMethod(
                regularization, self.diffusion_model, use_time_weight=rm.use_time_weight,
                sigma_x0=rm.sigma_x0, fixed_timestep=rm.fixed_timestep)

        B = mu.shape[0]
        mu = mu.float().clone().detach().to(self.device).requires_grad_(True)
        mu_true = mu_true.float().to(self.device)
        # K11: Adam + clamp in one HIP pass; the cosine schedule is a host scalar (no sync)
        optimizer = FusedAdamClamp(mu, lr=lr, clamp=(-1.0, 1.0))
        scheduler = CosineLR(lr, T_max=ts, eta_min=0.0)
        true_norm = v_normalize(mu_true).contiguous()           # metrics.py:24, loop-invariant
        loss_calc = LossCalculator(self.regularization_method)
        keys = ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")
        # per-iteration histories stay on the device; ONE copy to the host after the loop (the
        # reference syncs six times per iteration, inversion.py:97-111)
        hist_dev = torch.zeros(ts, len(keys), B, dtype=torch.float32, device=self.device)

        y = add_noise_to_seismic(y, noise_std, noise_type=noise_type, generator=None)
        y, mask = missing_trace(y, missing_number, return_mask=True, generator=None)
        y = y.to(self.device)
        mask = mask.to(self.device)

        shots = shot_slice(fwi_forward, y.shape[1])
        sharded = shots is not None and dist.is_available() and dist.is_initialized()
        if shots is not None:
            if sharded:   # global observation count, constant over the loop: one all-reduce
                nobs = mask.reshape(B, -1).sum(1).clamp(min=1.0)
                loss_calc.global_nobs = nobs
            y = y[:, shots[0]:shots[1]].contiguous()
            mask = mask[:, shots[0]:shots[1]].contiguous()
            if sharded and missing_number == 0:
                mask = None   # all ones: the kernel skips the mask stream
        elif missing_number == 0:
            mask = None

        pbar = tqdm(range(ts), desc="Optimizing", unit="step", disable=not self.show_progress)
        for it in pbar:
            if regularization == "diffusion":
                noise_x0 = torch.randn(mu.shape, device=mu.device, dtype=mu.dtype)
                x0_pred = mu + self.regularization_method.sigma_x0 * noise_x0
            else:
                x0_pred = mu
            v_in = x0_pred[:, :, 1:-1, 1:-1]
            if sharded:
                v_in = grad_all_reduce(v_in, process_group)
            predicted = fwi_forward(v_in)
            loss_obs = loss_calc.observation_loss(predicted, y, mask=mask)
            reg_loss, time_tensor = loss_calc.regularization_loss(x0_pred, generator=None)
            total_loss = loss_calc.total_loss(loss_obs, reg_loss, reg_lambda)

            optimizer.zero_grad()
            total_loss.sum().backward()
            optimizer.step()                       # + clamp_(-1, 1), inversion.py:87-90
            optimizer.lr = scheduler.step()

            with torch.no_grad():
                row = hist_dev[it]
                row[3:6] = fused_metrics(mu[:, :, 1:-1, 1:-1], true_norm)[[2, 0, 1]]   # ssim, mae, rmse
                obs_log = loss_obs.detach()
                if sharded:
                    obs_log = obs_log.clone()
                    dist.all_reduce(obs_log, group=process_group)
                row[0] = obs_log + reg_lambda * reg_loss.detach()
                row[1] = obs_log
                row[2] = reg_loss.detach()
            if self.show_progress:
                h = row.cpu().numpy()
                post = {"MAE": float(h[4].mean()), "RMSE": float(h[5].mean()), "SSIM": float(h[3].mean())}
                if time_tensor is not None:
                    post["t"] = int(round(time_tensor.float().mean().item()))
                pbar.set_postfix(post)

        check = getattr(fwi_forward, "check", None)   # persistent-kernel hand-off status (one sync)
        if callable(check):
            check()
        H = hist_dev.cpu().numpy()
        results = [{k: [H[t, j, i] for t in range(ts)] for j, k in enumerate(keys)} for i in range(B)]
        return mu[:, :, 1:-1, 1:-1], results
