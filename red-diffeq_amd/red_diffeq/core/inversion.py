"""InversionEngine (reference red_diffeq/core/inversion.py:12-129), same API and loop order.

Per iteration: [diffusion: eps_x0 ~ N(0,1); x0 = mu + sigma_x0 eps_x0] -> seis = fwi_forward(
x0[:, :, 1:-1, 1:-1]) -> L1 misfit -> regulariser -> backward (HIP adjoint) -> Adam -> clamp to
[-1,1] -> cosine LR step -> metrics.  RNG draw order matches the reference
(eps_x0, then the regulariser's t, then eps).

Shot-parallel inversion: when ``fwi_forward.shots`` covers a subset of the sources
and a torch.distributed process group is initialised, each rank models its shots only; the
misfit is normalised by the global observation count (computed from the full, replicated mask:
no communication); the data-term gradient is summed over ranks by ONE all-reduce inside backward
(``_GradAllReduce``); the regulariser, Adam and the metrics run replicated (identical seeds ->
identical draws on every rank).

Persistent-kernel failure (a neighbour hand-off or residency timeout of the single-launch FWI
kernels, reported through the plan's status word) is handled inside the loop, without a host sync
per iteration: see ``_FaultMonitor``.
"""
import os
import time
import warnings
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
from .metrics import MetricsCalculator


class _GradAllReduce(torch.autograd.Function):
    """Identity forward; backward sums the incoming gradient over the process group.  With a
    fault monitor, the local FWI status word rides along as one extra element of the same
    all-reduce, so every rank sees (and its Adam guard acts on) any rank's failed launch."""

    @staticmethod
    def forward(ctx, x, group, monitor):
        ctx.group, ctx.monitor = group, monitor
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        mon = ctx.monitor
        if mon is None:
            g = g.contiguous()
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=ctx.group)
            return g, None, None
        # the word rides as 0 / 1 (any status code, whatever its sign or bits, counts as a failure):
        # the sum is the number of failed ranks, exact in the gradient's dtype
        buf = torch.cat([g.reshape(-1), (mon.local_word() != 0).to(g.dtype)])
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=ctx.group)
        mon.global_word.copy_(buf[-1:])          # != 0 iff some rank's launch failed
        return buf[:-1].view_as(g), None, None


def grad_all_reduce(x, group=None, monitor=None):
    return _GradAllReduce.apply(x, group, monitor)


def shot_slice(fwi_forward, ns_total):
    """(start, stop) of the shots the operator models, or None when it models them all -- unless the
    caller asked for sharding explicitly (FWIForward(shots=...): `shots_explicit`), which keeps the
    sharded path (gradient all-reduce, global observation count) even for one rank holding every shot."""
    shots = getattr(fwi_forward, "shots", None)
    if shots is None or (shots[0] == 0 and shots[1] == ns_total and not getattr(fwi_forward, "shots_explicit", False)):
        return None
    return shots


class _FaultMonitor:
    """Stream-ordered watch over the FWI operator's status word (include/red_diffeq_fwi.h,
    rdq_fwi_set_status_buffer).

    * Adam guard: every iteration's fused Adam step reads the word on the device and is a no-op
      when it is set, so a gradient from a failed persistent launch never reaches mu or the Adam
      moments (the word is sticky: every later iteration is skipped too).
    * Detection: the word is copied asynchronously into pinned host memory after each step; at the
      start of iteration it the host reads iteration it-2's copy (already complete: the GPU is at
      most two iterations behind, so no extra stall), and everything at the end of the loop.
    * Recovery: the engine rewinds its host state (Adam step count, LR schedule, RNG) to the first
      failed iteration, switches the operator to its chunked kernels and replays from there.
    * Re-promotion: a failure is usually transient (another kernel sharing the chip made the
      resident grid wait), so after ``repromote_after`` clean iterations on the chunked kernels the
      operator goes back to the persistent ones (``FWIForward.restore_persistent``); each further
      failure doubles that wait.  More than ``max_recoveries`` failures raise.
    Sharded runs guard on the all-reduced word (``_GradAllReduce``), identical on every rank."""

    max_recoveries = 8

    def __init__(self, fwi_forward, ts, device, sharded, repromote_after=16):
        self.fwi = fwi_forward
        self.sharded = sharded
        self.host = torch.zeros(ts, dtype=torch.int32, pin_memory=True)
        self.events = [None] * ts
        self.global_word = torch.zeros(1, dtype=torch.int32, device=device)
        self._zero = torch.zeros(1, dtype=torch.int32, device=device)
        self.checked = 0
        self.recoveries = 0
        self.repromote_after = repromote_after
        self.repromote_at = None          # iteration at which the persistent kernels come back

    def local_word(self):
        w = self.fwi.status_word()
        return self._zero if w is None else w

    def guard(self):
        return self.global_word if self.sharded else self.local_word()

    def record(self, it):
        g = self.guard()
        self.host[it:it + 1].copy_(g, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(g.device))   # the stream the copy was issued on
        self.events[it] = ev

    def first_fault(self, upto):
        """First iteration <= upto whose guard copy is set (None if none); waits for those copies."""
        for j in range(self.checked, upto + 1):
            self.events[j].synchronize()
            if int(self.host[j]) != 0:
                return j
            self.checked = j + 1
        return None

    def recover(self, k, ts):
        if self.repromote_at is not None:
            raise RuntimeError(f"FWI kernels failed at iteration {k} on the chunked path")
        if self.recoveries >= self.max_recoveries:
            raise RuntimeError(f"persistent FWI launch failed {self.recoveries + 1} times (last at iteration {k})")
        wait = self.repromote_after << self.recoveries
        warnings.warn(f"persistent FWI launch failed at iteration {k} (status word set); the gradient was "
                      f"not applied; replaying from that iteration on the chunked kernels (persistent kernels "
                      f"again after {wait} iterations)", RuntimeWarning)
        self.fwi.fallback_to_chunked()
        self.global_word.zero_()
        self.host[k:].zero_()
        self.events[k:] = [None] * (ts - k)
        self.checked = k
        self.recoveries += 1
        self.repromote_at = k + wait

    def maybe_repromote(self, it):
        """At the start of iteration it: back to the persistent kernels once the wait is over."""
        if self.repromote_at is not None and it >= self.repromote_at:
            restore = getattr(self.fwi, "restore_persistent", None)
            if callable(restore):
                restore()
            self.repromote_at = None

    @property
    def recovered(self):
        return self.recoveries > 0


class _Progress:
    """The progress bar's MAE / RMSE / SSIM / t postfix without a host sync: an iteration's history
    row (and t) is copied asynchronously into pinned memory behind an event — at most every
    `interval` seconds (tqdm's own refresh period: a copy per iteration would cost the stream a
    device-to-host round trip each time) — and the bar shows the newest iteration whose copy has
    completed (event.query(), never a wait)."""

    interval = 0.1

    def __init__(self, ts, width, device):
        self.host = torch.zeros(ts, width + 1, dtype=torch.float32, pin_memory=True)
        self.events = [None] * ts
        self.shown = -1
        self.has_t = False
        self.last = -1e30

    def record(self, it, row, time_tensor):
        now = time.monotonic()
        if now - self.last < self.interval and it != len(self.events) - 1:
            return
        self.last = now
        n = row.numel()
        self.host[it, :n].copy_(row.reshape(-1), non_blocking=True)
        if time_tensor is not None:
            self.host[it, n:n + 1].copy_(time_tensor.float().mean().reshape(1), non_blocking=True)
            self.has_t = True
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(row.device))   # the copies' stream, not the current device's
        self.events[it] = ev

    def show(self, pbar, it, B):
        j = None
        lo = self.shown if self.shown < it else -1        # (after a rewind, it can be behind)
        for i in range(it, lo, -1):
            if self.events[i] is not None and self.events[i].query():
                j = i
                break
        if j is None:
            return
        self.shown = j
        h = self.host[j].numpy()
        row = h[:-1].reshape(-1, B)
        post = {"MAE": float(row[4].mean()), "RMSE": float(row[5].mean()), "SSIM": float(row[3].mean())}
        if self.has_t:
            post["t"] = int(round(float(h[-1])))
        pbar.set_postfix(post, refresh=False)


def k12_covers(ssim_loss):
    """True when the fused metrics kernel K12 (csrc/loop.hip) computes exactly the caller's SSIM: the
    reference's module (red_diffeq/utils/ssim.py:19-65) with its 11 x 11 Gaussian window (sigma 1.5,
    C1 = 0.01^2, C2 = 0.03^2).  K12 evaluates one single-channel model at a time, where size_average
    True and False give the same mean.  Any other module (another window, a subclass, a different
    metric) is called as the reference's MetricsCalculator calls it (core/metrics.py:13-46)."""
    if ssim_loss is None:
        return False
    t = type(ssim_loss)
    if t.__name__ != "SSIM" or t.__module__ != "red_diffeq.utils.ssim" or getattr(ssim_loss, "window_size", None) != 11:
        return False
    win = getattr(ssim_loss, "window", None)
    if win is not None:
        from ..utils.ssim import create_window
        ref = create_window(11, int(win.shape[0]))
        if tuple(win.shape) != tuple(ref.shape) or not torch.equal(win.detach().cpu().to(ref.dtype), ref):
            return False
    return True


class InversionEngine:

    # clean chunked iterations before a failed persistent operator is tried again (_FaultMonitor)
    repromote_after = 16

    def __init__(self, diffusion_model, ssim_loss: SSIM, regularization: Optional[str] = None,
                 use_time_weight: bool = False, sigma_x0: float = 0.0001, fixed_timestep: int = None,
                 show_progress: bool = True):
        self.diffusion_model = diffusion_model
        # optional list: when set, optimize() appends mu's interior (a device copy, after Adam and
        # the clamp) at every iteration — the per-iteration model trajectory, for parity tests
        self.model_trace = None
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
        # K12 computes MAE / RMSE / SSIM in one launch when the caller's ssim_loss is the reference's
        # SSIM; any other module is called per model as the reference's MetricsCalculator does
        metrics_calc = None if k12_covers(self.ssim_loss) else MetricsCalculator(self.ssim_loss)
        loss_calc = LossCalculator(self.regularization_method)
        keys = ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")
        # per-iteration histories stay on the device; ONE copy to the host after the loop (the
        # reference syncs six times per iteration, inversion.py:97-111)
        hist_dev = torch.zeros(ts, len(keys), B, dtype=torch.float32, device=self.device)
        # (mae, rmse, ssim) -> (ssim, mae, rmse) by a device index: indexing with a Python list
        # copies the list to the device synchronously, which held the host to the device once per
        # iteration (the next iteration's launches then started on an idle GPU)
        metric_order = torch.tensor([2, 0, 1], device=self.device)

        y = add_noise_to_seismic(y, noise_std, noise_type=noise_type, generator=None)
        y, mask = missing_trace(y, missing_number, return_mask=True, generator=None)
        y = y.to(self.device)
        mask = mask.to(self.device)

        shots = shot_slice(fwi_forward, y.shape[1])
        sharded = shots is not None and dist.is_available() and dist.is_initialized()
        if shots is not None:
            if sharded:   # global observation count from the full (replicated) mask: no communication
                nobs = mask.reshape(B, -1).sum(1).clamp(min=1.0)
                loss_calc.global_nobs = nobs
            y = y[:, shots[0]:shots[1]].contiguous()
            mask = mask[:, shots[0]:shots[1]].contiguous()
            if missing_number == 0:
                mask = None   # all ones: the kernel skips the mask stream (sharded or not)
        elif missing_number == 0:
            mask = None

        monitor = None
        if callable(getattr(fwi_forward, "status_word", None)) and mu.is_cuda:
            check = getattr(fwi_forward, "check", None)
            if callable(check):
                check()          # a failure before the loop (e.g. while making y) is the caller's
            monitor = _FaultMonitor(fwi_forward, ts, self.device, sharded, self.repromote_after)
        diffusion = regularization == "diffusion"
        overlap = diffusion and mu.is_cuda and not os.environ.get("RDQ_NO_OVERLAP")
        snaps = [None] * ts

        pbar = tqdm(total=ts, desc="Optimizing", unit="step", disable=not self.show_progress)
        prog = _Progress(ts, len(keys) * B, self.device) if self.show_progress and mu.is_cuda else None
        trace = self.model_trace
        it = 0
        while True:
            while it < ts:
                k = monitor.first_fault(it - 2) if monitor is not None else None
                if k is not None:
                    it = self._rewind(k, snaps, optimizer, scheduler, monitor, ts, pbar, trace, prog)
                    continue
                if monitor is not None:   # host state at the start of the iteration (for a replay)
                    monitor.maybe_repromote(it)
                    snaps[it] = (optimizer.t, scheduler.lr, scheduler.last_epoch, optimizer.lr,
                                 torch.cuda.get_rng_state(mu.device) if diffusion else None)
                if diffusion:
                    noise_x0 = torch.randn(mu.shape, device=mu.device, dtype=mu.dtype)
                    x0_pred = mu + self.regularization_method.sigma_x0 * noise_x0
                else:
                    x0_pred = mu
                v_in = x0_pred[:, :, 1:-1, 1:-1]
                if sharded:
                    v_in = grad_all_reduce(v_in, process_group, monitor)
                if overlap:
                    # the regulariser (U-Net forward, no dependence on the FWI operator) runs on a
                    # side stream beside the forward / adjoint: the persistent FWI grids leave CUs
                    # free, the U-Net's small kernels fill them.  RNG draws (t, eps) are taken here,
                    # in the reference's order (the operator draws nothing).
                    main = torch.cuda.current_stream(mu.device)
                    side = self._side_stream(mu.device)
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        reg_loss, time_tensor = loss_calc.regularization_loss(x0_pred, generator=None)
                    predicted = fwi_forward(v_in)
                    loss_obs = loss_calc.observation_loss(predicted, y, mask=mask)
                    # the data term's backward (the FWI adjoint) does not need the regulariser: it
                    # is run first, so the side stream's U-Net overlaps the adjoint too, and only the
                    # regulariser's (elementwise) backward waits for it.  d(obs + lambda reg) / d mu
                    # is accumulated as the same two-tensor sum as in one backward (bit for bit).
                    optimizer.zero_grad()
                    loss_obs.sum().backward()
                    main.wait_stream(side)
                    reg_loss.record_stream(main)
                    (reg_lambda * reg_loss).sum().backward()
                else:
                    predicted = fwi_forward(v_in)
                    loss_obs = loss_calc.observation_loss(predicted, y, mask=mask)
                    reg_loss, time_tensor = loss_calc.regularization_loss(x0_pred, generator=None)
                    total_loss = loss_calc.total_loss(loss_obs, reg_loss, reg_lambda)
                    optimizer.zero_grad()
                    total_loss.sum().backward()
                optimizer.step(guard=None if monitor is None else monitor.guard())   # + clamp_(-1, 1)
                optimizer.lr = scheduler.step()
                if monitor is not None:
                    monitor.record(it)

                with torch.no_grad():
                    row = hist_dev[it]
                    if metrics_calc is None:
                        row[3:6] = fused_metrics(mu[:, :, 1:-1, 1:-1], true_norm).index_select(0, metric_order)
                    else:
                        mae, rmse, ssim = metrics_calc.calculate(mu[:, :, 1:-1, 1:-1], mu_true)
                        row[3:6] = torch.stack([ssim, mae, rmse])
                    obs_log = loss_obs.detach()
                    if sharded:
                        obs_log = obs_log.clone()
                        dist.all_reduce(obs_log, group=process_group)
                    row[0] = obs_log + reg_lambda * reg_loss.detach()
                    row[1] = obs_log
                    row[2] = reg_loss.detach()
                    if trace is not None:
                        if len(trace) > it:          # replayed after a rewind
                            del trace[it:]
                        trace.append(mu.detach()[:, :, 1:-1, 1:-1].clone())
                if prog is not None:             # no per-iteration sync (the reference's .item()s)
                    prog.record(it, row, time_tensor)
                    prog.show(pbar, it, B)
                pbar.update(1)
                it += 1
            k = monitor.first_fault(ts - 1) if monitor is not None else None
            if k is None:
                break
            it = self._rewind(k, snaps, optimizer, scheduler, monitor, ts, pbar, trace, prog)
        pbar.close()

        H = hist_dev.cpu().numpy()
        results = [{k: [H[t, j, i] for t in range(ts)] for j, k in enumerate(keys)} for i in range(B)]
        return mu[:, :, 1:-1, 1:-1], results

    def _side_stream(self, device):
        streams = self.__dict__.setdefault("_streams", {})
        if device not in streams:
            streams[device] = torch.cuda.Stream(device=device)
        return streams[device]

    @staticmethod
    def _rewind(k, snaps, optimizer, scheduler, monitor, ts, pbar, trace=None, prog=None):
        """Restore the host state of iteration k (mu and the Adam moments are untouched: every step
        since the failure was skipped on the device) and switch to the chunked kernels."""
        monitor.recover(k, ts)
        if trace is not None:
            del trace[k:]
        if prog is not None:
            prog.events[k:] = [None] * (ts - k)
            prog.shown = min(prog.shown, k - 1)
        optimizer.t, scheduler.lr, scheduler.last_epoch, optimizer.lr, rng = snaps[k]
        if rng is not None:
            torch.cuda.set_rng_state(rng, optimizer.param.device)
        pbar.n = k
        return k
