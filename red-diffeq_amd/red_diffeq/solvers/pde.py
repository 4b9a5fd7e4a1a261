"""FWIForward — drop-in for the reference forward operator (red_diffeq/solvers/pde.py:6-93).

Same constructor, same ``ctx`` handling (including the in-place ``sx``/``gx`` mutation,
pde.py:16-24), same ``forward(v) -> seis`` contract: (B,1,H,W) fp32, possibly a non-contiguous
view, to (B, ns, ceil(nt/sample_temporal), ng') fp32, differentiable w.r.t. ``v``.

The compute is the MI355X HIP path (include/red_diffeq_fwi.h): coefficient fields (K3), the whole
time loop (stencil + periodic wrap + source injection + receiver sampling + history store) in one
persistent launch when the survey fits resident on the chip, else temporal-blocked launches of T
steps replayed from a cached hipGraph (K1), and a hand-written discrete adjoint (K2 + K4) as the
autograd backward of the custom operator torch.ops.red_diffeq.fwi (red_diffeq/ops.py) — where the
reference records a ~5 MB-per-shot-step autograd tape, this keeps one fp32 wavefield per step
(store-all history).
"""
import ctypes
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _hip
from .. import ops as _ops   # registers torch.ops.red_diffeq.*
from ..utils.data_trans import v_denormalize


def ricker(f, dt, nt):
    """Ricker wavelet, pde.py:26-36 (fp64; raises ValueError when nt is shorter than it)."""
    nw = 2.2 / f / dt
    nw = 2 * np.floor(nw / 2) + 1
    nc = np.floor(nw / 2)
    k = np.arange(nw)
    alpha = (nc - k) * f * dt * np.pi
    beta = alpha ** 2
    w0 = (1 - beta * 2) * np.exp(-beta)
    w = np.zeros(nt)
    w[:len(w0)] = w0
    return w


def adj_sr(sx, sz, gx, gz, dx, nbc):
    """Physical positions -> padded-grid indices, pde.py:54-59 (np.around: half to even)."""
    isx = np.around(sx / dx) + nbc
    isz = np.around(sz / dx) + nbc
    igx = np.around(gx / dx) + nbc
    igz = np.around(gz / dx) + nbc
    return isx.astype("int"), int(isz), igx.astype("int"), int(igz)


class FwiPlan:
    """Owns one C-ABI plan (uploaded geometry + cached hipGraphs) for one device."""

    def __init__(self, nz, nx, ctx, sample_temporal, isx, isz, igx, igz, wavelet, device):
        self.lib = _hip.lib()
        self.device = device
        self._isx = np.ascontiguousarray(isx, np.int32)
        self._igx = np.ascontiguousarray(igx, np.int32)
        self._wav = np.ascontiguousarray(wavelet, np.float64)
        g = _hip.FwiGeom(nz=nz, nx=nx, nbc=int(ctx["nbc"]), nt=int(ctx["nt"]), ns=len(self._isx),
                         ng=len(self._igx), sample_temporal=int(sample_temporal),
                         dx=float(ctx["dx"]), dt=float(ctx["dt"]), isz=int(isz), igz=int(igz),
                         isx=self._isx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                         igx=self._igx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                         wavelet=self._wav.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        self.ns, self.ng, self.nt, self.nz, self.nx = len(self._isx), len(self._igx), int(ctx["nt"]), nz, nx
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _hip.check(self.lib.rdq_fwi_plan_create(ctypes.byref(g), ctypes.byref(h)), "rdq_fwi_plan_create")
        self.handle = h
        self._sizes = {}
        self.persist_mode = 1                      # rdq_fwi_set_persistent mode (the C default: auto)
        self._saved_mode = None                    # mode before fallback_to_chunked (None: not fallen back)
        # status words in torch memory (caller-owned, rdq_fwi_set_status_buffer): word 0 != 0 once a
        # persistent launch gave up; read stream-ordered (Adam guard, async host copies)
        self.status_t = torch.zeros(64, dtype=torch.int32, device=device)
        _hip.check(self.lib.rdq_fwi_set_status_buffer(self.handle, _hip.ptr(self.status_t)),
                   "rdq_fwi_set_status_buffer")
        self.op_id = _ops.register_plan(self)      # integer handle for torch.ops.red_diffeq.fwi*

    def sizes(self, B):
        if B not in self._sizes:
            s = _hip.FwiSizes()
            _hip.check(self.lib.rdq_fwi_sizes(self.handle, B, ctypes.byref(s)), "rdq_fwi_sizes")
            self._sizes[B] = s
        return self._sizes[B]

    def set_graphs(self, enable):
        _hip.check(self.lib.rdq_fwi_set_graphs(self.handle, int(bool(enable))), "rdq_fwi_set_graphs")

    def set_variant(self, fwd_gen_coeffs=True, adj_exact=False, xcd_local=True, wide_chunked=True,
                    chunked_adj_fma=False):
        """fwd_gen_coeffs: chunked forward regenerates coefficients; adj_exact: persistent adjoint in
        the oracle's exact fp32 op order (bit-identical gA) instead of FMA contraction; xcd_local:
        persistent kernels keep whole slices on one XCD with L2-resident neighbour hand-offs;
        wide_chunked: chunked kernels on 128-column regions (two columns per lane) instead of 64;
        chunked_adj_fma: the wide chunked adjoint contracts its stencils into FMAs (opt-in; the default
        chunked adjoint keeps the oracle's exact order)."""
        flags = ((1 if fwd_gen_coeffs else 0) | (2 if adj_exact else 0) | (0 if xcd_local else 4)
                 | (0 if wide_chunked else 8) | (16 if chunked_adj_fma else 0))
        _hip.check(self.lib.rdq_fwi_set_variant(self.handle, flags), "rdq_fwi_set_variant")

    def set_wide_adj_steps(self, steps):
        """Time steps per launch of the wide chunked adjoint (1..6; 0 = the default, 5: fastest at
        configs[4] for both forms); set_tuning's adj_steps
        sets the persistent / narrow chunked adjoints' depth.  Results are identical for every depth."""
        _hip.check(self.lib.rdq_fwi_set_wide_adj_steps(self.handle, int(steps)), "rdq_fwi_set_wide_adj_steps")

    def set_wide_adj_shots(self, shots):
        """Shots per workgroup of the wide chunked adjoint (1..64; 0 = auto, the default: up to 16, from a
        cost model of launch rounds x (shots + a workgroup's fixed cost); the region's alpha / kappa are
        generated once for all of them).  Results are identical for every setting."""
        _hip.check(self.lib.rdq_fwi_set_wide_adj_shots(self.handle, int(shots)), "rdq_fwi_set_wide_adj_shots")

    def set_wide_fwd_steps(self, steps):
        """Time steps per launch of the wide chunked forward (1..6; 0 = set_tuning's fwd_steps).
        Results are identical for every depth."""
        _hip.check(self.lib.rdq_fwi_set_wide_fwd_steps(self.handle, int(steps)), "rdq_fwi_set_wide_fwd_steps")

    def set_wide_fwd_shots(self, shots):
        """Shots per workgroup of the wide chunked forward (as set_wide_adj_shots; 0 = auto)."""
        _hip.check(self.lib.rdq_fwi_set_wide_fwd_shots(self.handle, int(shots)), "rdq_fwi_set_wide_fwd_shots")

    def set_rows_per_wave(self, fwd_rows, adj_rows):
        """Rows per wave of the 64 x 96-region persistent kernels (forward 6 / 8 / 12 / 24, adjoint
        6 / 8 / 12; 6 is the default for both); results are the same for every choice."""
        _hip.check(self.lib.rdq_fwi_set_rows_per_wave(self.handle, int(fwd_rows), int(adj_rows)),
                   "rdq_fwi_set_rows_per_wave")

    def set_persistent(self, enable):
        """True / 1: persistent launches when they fit (small surveys in 64 x 64 regions of 16 waves x
        4 rows, else 64 x 96 regions, else 64 x 64 of 8 waves x 8 rows); 16 / 12 / 8: persistent with
        that region class only; False / 0: chunked launches.  Results are identical in every mode.
        -1 (fault-path tests): persistent launches oversubscribed past residency, which fail.
        A direct call during an engine fallback (FWIForward.fallback_to_chunked) replaces the mode the
        restore would bring back."""
        mode = int(enable) if not isinstance(enable, bool) else int(enable)
        self._set_mode(mode)
        if self._saved_mode is not None:
            self._saved_mode = mode

    def _set_mode(self, mode):
        _hip.check(self.lib.rdq_fwi_set_persistent(self.handle, mode), "rdq_fwi_set_persistent")
        self.persist_mode = mode

    def status(self, stream=None):
        """Synchronise and raise if a persistent launch's neighbour hand-off timed out."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        _hip.check(self.lib.rdq_fwi_status(self.handle, ctypes.c_void_p(stream)), "rdq_fwi_status")

    def debug_words(self):
        """[status, per-XCD workgroup counts of the last persistent launch] (synchronises)."""
        out = (ctypes.c_uint32 * 32)()
        _hip.check(self.lib.rdq_fwi_debug_words(self.handle, out), "rdq_fwi_debug_words")
        return int(out[0]), [int(v) for v in out[1:7]], [int(v) for v in out[16:24]]

    def launch_info(self, B):
        """{'fwd_persistent', 'adj_persistent', 'fwd_class' / 'adj_class' (persistent region class: 16 /
        12 / 8, 0 = chunked), 'fwd_T', 'adj_T', 'fwd_launches', 'adj_launches'} of a
        call with batch B (launches: time-loop kernel launches per call)."""
        out = (ctypes.c_int32 * 6)()
        _hip.check(self.lib.rdq_fwi_launch_info(self.handle, int(B), out), "rdq_fwi_launch_info")
        return {"fwd_persistent": bool(out[0]), "adj_persistent": bool(out[1]),
                "fwd_class": int(out[0]), "adj_class": int(out[1]), "fwd_T": int(out[2]),
                "adj_T": int(out[3]), "fwd_launches": int(out[4]), "adj_launches": int(out[5])}

    def set_sweep_delay(self, fwd_ticks, adj_ticks):
        """Persistent kernels: 10 ns ticks between an epoch's publish and its first hand-off pass."""
        _hip.check(self.lib.rdq_fwi_set_sweep_delay(self.handle, int(fwd_ticks), int(adj_ticks)),
                   "rdq_fwi_set_sweep_delay")

    def wide_info(self, B):
        """{'chains', 'fwd_spw', 'adj_spw', 'chain0_shots'}: the wide chunked kernels' concurrent launch
        chains and shots per workgroup of chain 0's full-depth forward / adjoint launches for batch B
        (the automatic choice unless set_wide_*_shots fixed one)."""
        out = (ctypes.c_int32 * 4)()
        _hip.check(self.lib.rdq_fwi_wide_info(self.handle, int(B), out), "rdq_fwi_wide_info")
        return {"chains": int(out[0]), "fwd_spw": int(out[1]), "adj_spw": int(out[2]), "chain0_shots": int(out[3])}

    def set_profile(self, enable):
        _hip.check(self.lib.rdq_fwi_set_profile(self.handle, int(bool(enable))), "rdq_fwi_set_profile")

    def read_profile(self):
        """Per-wave average phase times (us) of the persistent kernels since the last read."""
        out = (ctypes.c_uint64 * 12)()
        _hip.check(self.lib.rdq_fwi_read_profile(self.handle, out), "rdq_fwi_read_profile")
        res = {}
        for name, o in (("fwd", 0), ("adj", 6)):
            n = max(int(out[o + 3]), 1)
            res[name] = {"wait_us": out[o] / n / 100.0, "steps_us": out[o + 1] / n / 100.0,
                         "publish_us": out[o + 2] / n / 100.0, "waves": int(out[o + 3]),
                         "first_pass_us": out[o + 4] / n / 100.0, "passes": out[o + 5] / n}
        return res

    def profile_waves(self, adj):
        """(blocks*16, 3) per-wave {hand-off, steps, publish} us of the last read_profile()."""
        n = 4096 * 16 * 3
        out = (ctypes.c_uint64 * n)()
        _hip.check(self.lib.rdq_fwi_profile_waves(self.handle, int(bool(adj)), out, n), "rdq_fwi_profile_waves")
        return np.frombuffer(out, dtype=np.uint64).reshape(-1, 3).astype(np.float64) / 100.0

    def set_tuning(self, fwd_steps, adj_steps, chains=0):
        """Blocking depths (1..4) and concurrent launch chains of the chunked kernels (0 = auto)."""
        _hip.check(self.lib.rdq_fwi_set_tuning(self.handle, int(fwd_steps), int(adj_steps), int(chains)),
                   "rdq_fwi_set_tuning")

    def __del__(self):
        try:
            _ops.unregister_plan(getattr(self, "op_id", -1))
        except Exception:          # interpreter shutdown: module globals already torn down
            pass
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.rdq_fwi_plan_destroy(h)
            except Exception:
                pass
            self.handle = None

    # ---- the C ABI entry points as torch.ops.red_diffeq operators (red_diffeq/ops.py) ----
    def coeffs(self, v, vel_mode):
        return torch.ops.red_diffeq.fwi_coeffs(v, self.op_id, vel_mode)

    def forward(self, coeffs, B, keep_history):
        seis, hist = torch.ops.red_diffeq.fwi_forward(coeffs, self.op_id, B, bool(keep_history))
        return seis, (hist if keep_history else None)

    def adjoint(self, coeffs, hist, dseis, B):
        return torch.ops.red_diffeq.fwi_adjoint(coeffs, hist, dseis, self.op_id, B)

    def finalize(self, coeffs, vstat, gA, gk, gb, B, vel_mode):
        return torch.ops.red_diffeq.fwi_grad_finalize(coeffs, vstat, gA, gk, gb, self.op_id, B, vel_mode)


class FWIForward(nn.Module):
    """Drop-in for red_diffeq.solvers.pde.FWIForward (pde.py:6-93)."""

    def __init__(self, ctx, device, sample_temporal=1, sample_spatial=1.0, normalize=True,
                 v_denorm_func=None, s_norm_func=None, shots=None):
        super().__init__()
        self.device = device
        self.normalize = normalize
        if normalize:
            self.v_denorm_func = v_denorm_func
            self.s_norm_func = s_norm_func
        self.sample_temporal = sample_temporal
        if "sx" not in ctx.keys():
            ctx["sx"] = np.linspace(0, ctx["n_grid"] - 1, num=ctx["ns"]) * ctx["dx"]
        else:
            ctx["sx"] = np.array(ctx["sx"]) * ctx["dx"]
        if "gx" not in ctx.keys():
            ctx["gx"] = np.linspace(0, ctx["n_grid"] - 1, num=int(sample_spatial * ctx["ng"])) * ctx["dx"]
        else:
            ctx["gx"] = np.array(ctx["gx"]) * ctx["dx"]
        self.ctx = ctx
        # shot-parallel sharding: this operator models only shots[start:stop]
        self.shots = (0, len(ctx["sx"])) if shots is None else (int(shots[0]), int(shots[1]))
        self.shots_explicit = shots is not None
        self._plans = {}
        self._last = None
        self._fallen_back = False      # between fallback_to_chunked() and restore_persistent()

    # --- reference helpers kept with their signatures -------------------------------------
    def ricker(self, f, dt, nt):
        return ricker(f, dt, nt)

    def adj_sr(self, sx, sz, gx, gz, dx, nbc):
        return adj_sr(sx, sz, gx, gz, dx, nbc)

    def get_Abc(self, vp, nbc, dx):
        """Sponge damping field of a padded velocity (pde.py:38-52), for inspection only.

        The hot path never calls this: the same profile is fused into the HIP coefficient kernel
        (rdq_fwi_coeffs).  Columns overwrite rows, so the corners take the column profile."""
        dimrange = 1.0 * torch.unsqueeze(torch.arange(nbc, device=vp.device), dim=-1)
        velmin, _ = torch.min(vp.view(vp.shape[0], -1), dim=-1)
        a = (nbc - 1) * dx
        kappa = (3.0 * velmin * np.log(10000000.0) / (2.0 * a)).unsqueeze(0).expand(nbc, -1)
        prof = (kappa * (dimrange * dx / a) ** 2).permute(1, 0).unsqueeze(1)   # (B,1,nbc)
        damp = torch.zeros_like(vp)
        H, W = vp.shape[-2:]
        damp[:, :, :nbc, :] = torch.flip(prof, dims=[-1]).unsqueeze(-1).expand(-1, -1, -1, W)
        damp[:, :, H - nbc:, :] = prof.unsqueeze(-1).expand(-1, -1, -1, W)
        damp[:, :, :, :nbc] = torch.flip(prof, dims=[-1]).unsqueeze(-2).expand(-1, -1, H, -1)
        damp[:, :, :, W - nbc:] = prof.unsqueeze(-2).expand(-1, -1, H, -1)
        return damp

    # --- HIP path --------------------------------------------------------------------------
    def _plan(self, nz, nx, device):
        key = (nz, nx, device.index)
        if key not in self._plans:
            c = self.ctx
            isx, isz, igx, igz = adj_sr(np.asarray(c["sx"]), c["sz"], np.asarray(c["gx"]), c["gz"],
                                        c["dx"], c["nbc"])
            isx = isx[self.shots[0]:self.shots[1]]
            if len(isx) == 0:
                raise ValueError("empty shot range")
            self._plans[key] = FwiPlan(nz, nx, c, self.sample_temporal, isx, isz, igx, igz,
                                       ricker(c["f"], c["dt"], c["nt"]), device)
            if os.environ.get("RDQ_NO_XCD_LOCAL"):       # A/B switches (tools/, experiments)
                self._plans[key].set_variant(xcd_local=False)
            if os.environ.get("RDQ_NO_GRAPHS"):
                self._plans[key].set_graphs(False)
            if os.environ.get("RDQ_ROWS_PER_WAVE"):          # "fwd,adj" (tools/ab_rw.sh, red_loop A/B)
                self._plans[key].set_rows_per_wave(*[int(x) for x in os.environ["RDQ_ROWS_PER_WAVE"].split(",")])
            if self._fallen_back:     # created during a fallback: chunked until restore_persistent()
                plan = self._plans[key]
                plan._saved_mode = plan.persist_mode
                plan._set_mode(0)
        return self._plans[key]

    def _fused_denorm(self):
        return self.normalize and self.v_denorm_func is v_denormalize

    def forward(self, v):
        _hip.require_device(v)
        if v.dim() != 4 or v.shape[1] != 1:
            raise ValueError(f"expected v of shape (B,1,H,W), got {tuple(v.shape)}")
        if v.dtype != torch.float32:
            v = v.float()
        if self._fused_denorm():
            vel_mode = 0                      # denormalisation fused into K3 / K4
        else:
            if self.normalize:
                v = self.v_denorm_func(v)     # arbitrary user callable: autograd through torch
            vel_mode = 1
        plan = self._plan(v.shape[2], v.shape[3], v.device)
        self._last = plan
        keep = bool(v.requires_grad and torch.is_grad_enabled())
        s = torch.ops.red_diffeq.fwi(v, plan.op_id, vel_mode, keep)[0]   # backward: K2 + K4 (ops.py)
        return self.s_norm_func(s) if self.normalize else s

    def check(self):
        """Raise if a persistent kernel's neighbour hand-off timed out since the last check
        (synchronises the current stream)."""
        for plan in self._plans.values():
            plan.status()

    def status_word(self):
        """Device int32 view (1,) of the status word of the plan the last call used (None before the
        first call): non-zero once a persistent launch gave up.  Stream-ordered, no sync."""
        return None if self._last is None else self._last.status_t[:1]

    def fallback_to_chunked(self):
        """After a persistent-launch failure: every plan runs the chunked (non-resident) kernels until
        restore_persistent(), and the status words are cleared (stream-ordered).  Each plan's mode
        is saved once (a second fallback before the restore keeps the first saved mode); plans created
        while fallen back (a new grid shape) start chunked too (_plan)."""
        self._fallen_back = True
        for plan in self._plans.values():
            if plan._saved_mode is None:
                plan._saved_mode = plan.persist_mode
            plan._set_mode(0)
            plan.status_t.zero_()

    def restore_persistent(self):
        """Back to the persistent kernels (where they fit) after fallback_to_chunked(): the engine
        re-promotes after a number of clean iterations (core/inversion.py _FaultMonitor).  Each plan
        gets back the mode it had before the fallback: a plan pinned to the chunked kernels (0) or to
        one region class (8 / 12 / 16) keeps it; the fault-path test mode (-1) comes back as auto (1).
        A plan whose mode was set directly (set_persistent) during the fallback keeps that mode."""
        self._fallen_back = False
        for plan in self._plans.values():
            mode = plan._saved_mode
            if mode is None:
                continue                           # never fell back: nothing to restore
            plan._saved_mode = None
            plan._set_mode(1 if mode == -1 else mode)

    def coefficients(self, v):
        """Debug/inspection: the K3 fields (alpha, temp1, temp2, kappa, beta, v) on the padded grid."""
        _hip.require_device(v)
        plan = self._plan(v.shape[2], v.shape[3], v.device)
        v = v.float()
        if self.normalize and not self._fused_denorm():
            v = self.v_denorm_func(v)
        coeffs, vstat = plan.coeffs(v, 0 if self._fused_denorm() else 1)
        sz = plan.sizes(v.shape[0])
        f = coeffs[:6 * v.shape[0] * sz.Hp * sz.ld].view(6, v.shape[0], sz.Hp, sz.ld)[..., :sz.Wp]
        return dict(zip(("alpha", "temp1", "temp2", "kappa", "beta", "v"), f.unbind(0)))
