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
from ..utils.ssim import SSIM
from .losses import LossCalculator
from .metrics import MetricsCalculator


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
        optimizer = torch.optim.Adam([mu], lr=lr)
        scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=ts, eta_min=0.0)
        metrics_calc = MetricsCalculator(self.ssim_loss)
        loss_calc = LossCalculator(self.regularization_method)
        hist = {k: [] for k in ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")}

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
        for _ in pbar:
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

            optimizer.zero_grad(set_to_none=True)
            total_loss.sum().backward()
            optimizer.step()
            with torch.no_grad():
                mu.data.clamp_(-1, 1)
            scheduler.step()

            mae, rmse, ssim = metrics_calc.calculate(mu[:, :, 1:-1, 1:-1], mu_true)
            obs_log = loss_obs.detach()
            if sharded:
                obs_log = obs_log.clone()
                dist.all_reduce(obs_log, group=process_group)
            tot_log = obs_log + reg_lambda * reg_loss.detach()
            hist["total_losses"].append(tot_log.cpu().numpy())
            hist["obs_losses"].append(obs_log.cpu().numpy())
            hist["reg_losses"].append(reg_loss.detach().cpu().numpy())
            hist["ssim"].append(ssim.cpu().numpy())
            hist["mae"].append(mae.cpu().numpy())
            hist["rmse"].append(rmse.cpu().numpy())
            if self.show_progress:
                post = {"MAE": float(hist["mae"][-1].mean()), "RMSE": float(hist["rmse"][-1].mean()),
                        "SSIM": float(hist["ssim"][-1].mean())}
                if time_tensor is not None:
                    post["t"] = int(round(time_tensor.float().mean().item()))
                pbar.set_postfix(post)

        n = len(hist["total_losses"])
        results = [{k: [hist[k][t][i] for t in range(n)] for k in hist} for i in range(B)]
        return mu[:, :, 1:-1, 1:-1], results
