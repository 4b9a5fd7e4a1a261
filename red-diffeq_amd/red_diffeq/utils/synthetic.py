"""Synthetic OpenFWI-shaped velocity models.

The OpenFWI datasets are not available offline, so the benchmarks and parity tests use seeded
NumPy models in the velocity range that ``v_normalize`` assumes (1500-4500 m/s,
red_diffeq/utils/data_trans.py:8-10 in the reference):

* ``flatvel``    - FlatVel-A-like: 3-5 flat layers, velocity increasing with depth.
* ``curvevel``   - CurveVel-A-like: sinusoidally curved interfaces, increasing with depth.
* ``curvefault`` - CurveFault-B-like: curved layers, one fault offset, non-monotone velocities.

This module deliberately has no package-relative imports so that fixture generators can load it
by file path.
"""
import numpy as np

VMIN, VMAX = 1500.0, 4500.0


def _layer_velocities(rng, n, monotone):
    v = np.sort(rng.uniform(VMIN, VMAX, size=n)) if monotone else rng.uniform(VMIN, VMAX, size=n)
    return v


def flatvel(nz=70, nx=70, seed=8888):
    rng = np.random.default_rng(seed)
    nl = int(rng.integers(3, 6))
    m = max(2, nz // 14)
    depths = np.sort(rng.choice(np.arange(m, nz - m), size=nl - 1, replace=False))
    vel = _layer_velocities(rng, nl, monotone=True)
    v = np.empty((nz, nx), np.float32)
    bounds = [0, *depths.tolist(), nz]
    for i in range(nl):
        v[bounds[i]:bounds[i + 1], :] = vel[i]
    return v


def _curved_layers(rng, nz, nx, nl, monotone, fault=False):
    x = np.arange(nx)
    m = max(2, nz // 9)
    base = np.sort(rng.choice(np.arange(m, nz - m), size=nl - 1, replace=False)).astype(np.float64)
    amp = rng.uniform(2.0, 6.0)
    period = rng.uniform(0.5, 1.5) * nx
    phase = rng.uniform(0, 2 * np.pi)
    curve = amp * np.sin(2 * np.pi * x / period + phase)
    vel = _layer_velocities(rng, nl, monotone)
    z = np.arange(nz)[:, None].astype(np.float64)
    shift = np.zeros(nx)
    if fault:
        xf = int(rng.integers(nx // 4, 3 * nx // 4))
        shift[xf:] = rng.uniform(4.0, 10.0)
    layer = np.zeros((nz, nx), np.int64)
    for d in base:
        layer += (z >= d + curve[None, :] + shift[None, :]).astype(np.int64)
    return vel[layer].astype(np.float32)


def curvevel(nz=70, nx=70, seed=8888):
    rng = np.random.default_rng(seed)
    return _curved_layers(rng, nz, nx, int(rng.integers(3, 6)), monotone=True)


def curvefault(nz=70, nx=70, seed=8888):
    rng = np.random.default_rng(seed)
    return _curved_layers(rng, nz, nx, int(rng.integers(3, 6)), monotone=False, fault=True)


FAMILIES = {"flatvel": flatvel, "curvevel": curvevel, "curvefault": curvefault}


def make_model(family="flatvel", nz=70, nx=70, seed=8888, batch=1):
    """Return a (batch, 1, nz, nx) float32 velocity array in m/s."""
    fn = FAMILIES[family]
    return np.stack([fn(nz, nx, seed + b)[None] for b in range(batch)]).astype(np.float32)
