"""Diagnose the persistent kernels' XCD-local assignment: run the bench step sequence (forward +
L1 + TV + backward + Adam) and print the status word and per-XCD workgroup counts per step.
python tools/xcd_diag.py [--steps 20] [--no-xcd]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.core.losses import l1_misfit  # noqa: E402
from red_diffeq.regularization.benchmark import total_variation_loss  # noqa: E402
from red_diffeq.solvers.pde import FWIForward  # noqa: E402
from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize  # noqa: E402
from red_diffeq.utils.synthetic import make_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--ns", type=int, default=8)
ap.add_argument("--no-xcd", action="store_true")
ap.add_argument("--no-graphs", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
ctx = dict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=a.ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
vt = torch.from_numpy(make_model("flatvel", 70, 70, batch=1))
plan = fwi._plan(70, 70, dev)
plan.set_variant(xcd_local=not a.no_xcd)
if a.no_graphs:
    plan.set_graphs(False)
with torch.no_grad():
    y = fwi(v_normalize(vt).to(dev))
print("after observed:", plan.debug_words(), flush=True)
mu = torch.nn.functional.pad(v_normalize(vt) * 0.9, (1, 1, 1, 1)).to(dev).requires_grad_(True)
opt = torch.optim.Adam([mu], lr=0.03)
for i in range(a.steps):
    loss = l1_misfit(fwi(mu[:, :, 1:-1, 1:-1]), y) + 0.01 * total_variation_loss(mu)
    opt.zero_grad()
    loss.sum().backward()
    opt.step()
    print(i, plan.debug_words(), flush=True)

# ---- InversionEngine path (bench loop_wallclock)
import types  # noqa: E402
from red_diffeq.core.inversion import InversionEngine  # noqa: E402
from red_diffeq.utils.ssim import SSIM  # noqa: E402
from red_diffeq.utils.data_trans import prepare_initial_model  # noqa: E402
eng = InversionEngine(types.SimpleNamespace(device=dev), SSIM(), regularization="tv", show_progress=False)
mu0 = torch.nn.functional.pad(prepare_initial_model(vt, "smoothed", sigma=10.0), (1, 1, 1, 1))
for rep in range(4):
    try:
        eng.optimize(mu0, vt, y, fwi, ts=3, lr=0.03, reg_lambda=0.01, regularization="tv")
        print("optimize", rep, "ok", plan.debug_words(), flush=True)
    except RuntimeError as e:
        print("optimize", rep, "FAILED", e, plan.debug_words(), flush=True)
