"""Sensitivity of the DiffusionFWI trajectory (tests/test_gpu_dfwi.py, fixture dfwi_small) to
fp32-ulp-level changes of the U-Net output: the same run with eps_hat scaled by (1 + k*1e-7) for a
few k, against the unperturbed run and the reference fixture.  Prints the per-step obs-loss spread
(the floor an implementation with a different summation order cannot be held below)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import ctx_of, load_golden  # noqa: E402
from test_gpu_dfwi import _diffusion  # noqa: E402


def run(scale):
    from diffusion_bench import DiffusionFWI
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
    from red_diffeq.utils.ssim import SSIM
    cuda = torch.device("cuda:0")
    z = load_golden("dfwi_small")
    fwi = FWIForward(dict(ctx_of(z)), cuda, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    diff = _diffusion(cuda)
    fwd = diff.model.forward
    diff.model.forward = lambda *a, **k: fwd(*a, **k) * scale
    bench = DiffusionFWI(diff, fwi, SSIM())
    mu, hist = bench.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]),
                              torch.from_numpy(z["y"]).to(cuda), fwi, ts=3, diffusion_ts=4, lr=0.03)
    return np.array(hist[0]["obs_losses"]), z["base_obs"], mu.cpu().numpy(), z["base_mu"]

def where_diff():
    """Cells where the final model differs from the reference fixture by > 0.01."""
    base, ref, mu, mu_ref = run(1.0)
    d = np.abs(mu - mu_ref)[0, 0]
    idx = np.argwhere(d > 0.01)
    return {"n": int(len(idx)), "cells": idx[:20].tolist(), "ours": mu[0, 0][d > 0.01][:20].tolist(),
            "ref": mu_ref[0, 0][d > 0.01][:20].tolist(), "shape": list(d.shape)}


if __name__ == "__main__" and "--where" in sys.argv:
    print(json.dumps(where_diff()))
elif __name__ == "__main__":
    base, ref, mu, mu_ref = run(1.0)
    out = {"ref": ref.tolist(), "ours": base.tolist(), "rel_vs_ref": (np.abs(base - ref) / np.abs(ref)).tolist(),
           "mu_maxabs_vs_ref": float(np.abs(mu - mu_ref).max())}
    for k in (1, -1, 3):
        o, _, m, _ = run(1.0 + k * 1e-7)
        out[f"rel_perturbed_{k}e-7"] = (np.abs(o - base) / np.abs(base)).tolist()
        out[f"mu_maxabs_perturbed_{k}e-7"] = float(np.abs(m - mu).max())
    print(json.dumps(out))

