"""ORACLE — TEST INFRASTRUCTURE ONLY.

Python side of the CPU restatement of red-diffeq's FWI hot path.  Importable only from tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker; the product package
(red-diffeq_amd/red_diffeq) never imports it.

* numpy restatements of the host geometry: ``ricker`` (red_diffeq/solvers/pde.py:26-36),
  source/receiver placement (pde.py:16-23 + ``adj_sr`` pde.py:54-59), the L1 observation loss
  and its adjoint source (red_diffeq/core/losses.py:14-41).
* ctypes bindings of ``fwi_oracle.c`` (forward, adjoint, gradient finalize) — built by
  ``make -C oracle``.

Pinned against tests/golden/*.npz, which tests/golden/make_golden.py produced by running the
reference itself in the build container.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libfwi_oracle.so")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


# ---------------------------------------------------------------------------- host geometry
def ricker(f, dt, nt):
    """pde.py:26-36 (float64)."""
    nw = 2.2 / f / dt
    nw = 2 * np.floor(nw / 2) + 1
    nc = np.floor(nw / 2)
    k = np.arange(nw)
    a = (nc - k) * f * dt * np.pi
    b = a ** 2
    w0 = (1 - b * 2) * np.exp(-b)
    w = np.zeros(nt)
    w[:len(w0)] = w0          # raises like the reference when nt < len(w0)
    return w


def geometry(ctx, sample_spatial=1.0):
    """Source / receiver grid indices: pde.py:16-23 then adj_sr pde.py:54-59."""
    dx, nbc = ctx["dx"], ctx["nbc"]
    sx = (np.array(ctx["sx"]) * dx) if "sx" in ctx else np.linspace(0, ctx["n_grid"] - 1, num=ctx["ns"]) * dx
    gx = (np.array(ctx["gx"]) * dx) if "gx" in ctx else \
        np.linspace(0, ctx["n_grid"] - 1, num=int(sample_spatial * ctx["ng"])) * dx
    isx = (np.around(sx / dx) + nbc).astype(np.int64)
    igx = (np.around(gx / dx) + nbc).astype(np.int64)
    isz = int(np.around(ctx["sz"] / dx) + nbc)
    igz = int(np.around(ctx["gz"] / dx) + nbc)
    return isx, isz, igx, igz


def l1_loss(pred, y, mask=None):
    """losses.py:14-41: per-model L1, plus dL/dpred = sign(pred - y) * mask / n_obs."""
    pred = pred.astype(np.float32)
    y = y.astype(np.float32)
    B = pred.shape[0]
    d = np.abs(y - pred)
    if mask is None:
        nobs = np.full(B, np.float32(np.prod(pred.shape[1:])))
        m = np.ones_like(pred)
    else:
        m = mask.astype(np.float32)
        nobs = np.maximum(m.reshape(B, -1).sum(1, dtype=np.float64), 1.0).astype(np.float32)
    loss = (d * m).reshape(B, -1).sum(1, dtype=np.float64) / nobs
    dseis = np.sign(pred - y) * m / nobs.reshape((B,) + (1,) * (pred.ndim - 1))
    return loss.astype(np.float32), dseis.astype(np.float32)


# ---------------------------------------------------------------------------- C bindings
class _Geom(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("ns", ctypes.c_int), ("ng", ctypes.c_int), ("nt", ctypes.c_int),
                ("nz", ctypes.c_int), ("nx", ctypes.c_int), ("nbc", ctypes.c_int), ("st", ctypes.c_int),
                ("dx", ctypes.c_float), ("dt", ctypes.c_float), ("isz", ctypes.c_int), ("igz", ctypes.c_int),
                ("isx", ctypes.POINTER(ctypes.c_int)), ("igx", ctypes.POINTER(ctypes.c_int)),
                ("wavelet", ctypes.POINTER(ctypes.c_double))]


_libs = {}


def lib(variant=""):
    """The oracle library; variant "fma" is the FMA-contracted build (ensemble member only)."""
    if variant not in _libs:
        path = LIB if not variant else LIB.replace(".so", "_" + variant + ".so")
        if not os.path.exists(path):
            build()
        _libs[variant] = ctypes.CDLL(path)
    return _libs[variant]


def _p(a, t=ctypes.c_float):
    return a.ctypes.data_as(ctypes.POINTER(t))


class OracleFWI:
    """CPU restatement of FWIForward (normalize=True, v_denormalize, s_normalize_none)."""

    def __init__(self, ctx, B, sample_temporal=1, sample_spatial=1.0, variant=""):
        self.ctx = dict(ctx)
        self.variant = variant
        isx, isz, igx, igz = geometry(ctx, sample_spatial)
        self.isx = np.ascontiguousarray(isx, np.int32)
        self.igx = np.ascontiguousarray(igx, np.int32)
        self.wav = np.ascontiguousarray(ricker(ctx["f"], ctx["dt"], ctx["nt"]), np.float64)
        nz = ctx.get("nz", None)
        self.g = _Geom(B=B, ns=len(isx), ng=len(igx), nt=int(ctx["nt"]), nz=0, nx=0,
                       nbc=int(ctx["nbc"]), st=int(sample_temporal), dx=float(ctx["dx"]),
                       dt=float(ctx["dt"]), isz=isz, igz=igz, isx=_p(self.isx, ctypes.c_int),
                       igx=_p(self.igx, ctypes.c_int), wavelet=_p(self.wav, ctypes.c_double))
        del nz

    def _shape(self, vn):
        B, _, nz, nx = vn.shape
        self.g.B, self.g.nz, self.g.nx = B, nz, nx
        nbc = self.g.nbc
        return B, nz + 2 * nbc, nx + 2 * nbc

    @property
    def nrec(self):
        return (self.g.nt + self.g.st - 1) // self.g.st

    def coeffs(self, vnorm):
        vn = np.ascontiguousarray(vnorm, np.float32)
        B, Hp, Wp = self._shape(vn)
        L = lib(self.variant)
        vpad = np.empty((B, Hp, Wp), np.float32)
        L.oracle_vpad(ctypes.byref(self.g), _p(vn), _p(vpad))
        f = {k: np.empty((B, Hp, Wp), np.float32) for k in ("alpha", "temp1", "temp2", "kappa", "beta")}
        vmin = np.empty(B, np.float32)
        amin = np.empty(B, np.int64)
        L.oracle_coeffs(ctypes.byref(self.g), _p(vpad), _p(f["alpha"]), _p(f["temp1"]), _p(f["temp2"]),
                        _p(f["kappa"]), _p(f["beta"]), _p(vmin), _p(amin, ctypes.c_int64))
        f.update(vpad=vpad, vmin=vmin, argmin=amin)
        return f

    def forward(self, vnorm, keep_history=False):
        c = self.coeffs(vnorm)
        B, Hp, Wp = c["vpad"].shape
        g = self.g
        seis = np.zeros((B, g.ns, self.nrec, g.ng), np.float32)
        hist = np.empty((g.nt + 2, B, g.ns, Hp, Wp), np.float32) if keep_history else None
        lib(self.variant).oracle_forward(ctypes.byref(g), _p(c["alpha"]), _p(c["temp1"]), _p(c["temp2"]),
                             _p(c["beta"]), _p(seis), _p(hist) if keep_history else None)
        if keep_history:
            c["hist"] = hist
        return seis, c

    def adjoint(self, c, dseis):
        g = self.g
        B, Hp, Wp = c["vpad"].shape
        dseis = np.ascontiguousarray(dseis, np.float32)
        gA = np.empty((B, Hp, Wp), np.float32)
        gK = np.empty(B, np.float64)
        gb = np.empty((B, g.ns), np.float32)
        lib(self.variant).oracle_adjoint(ctypes.byref(g), _p(c["alpha"]), _p(c["temp1"]), _p(c["temp2"]),
                             _p(c["kappa"]), _p(c["hist"]), _p(dseis), _p(gA), _p(gK, ctypes.c_double), _p(gb))
        return gA, gK, gb

    def finalize(self, c, gA, gK, gb):
        g = self.g
        B = gA.shape[0]
        out = np.empty((B, 1, g.nz, g.nx), np.float32)
        lib(self.variant).oracle_grad_finalize(ctypes.byref(g), _p(c["vpad"]), _p(gA), _p(gK, ctypes.c_double),
                                   _p(gb), _p(c["vmin"]), _p(c["argmin"], ctypes.c_int64), _p(out))
        return out

    def gradient(self, vnorm, dseis):
        """dL/dv_norm given dL/dseis (the autograd path of the reference)."""
        _, c = self.forward(vnorm, keep_history=True)
        gA, gK, gb = self.adjoint(c, dseis)
        return self.finalize(c, gA, gK, gb)
