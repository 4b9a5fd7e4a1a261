"""One configs[4]-grid forward + adjoint (chunked kernels) for counter / trace runs:
python tools/large_once.py [--ns 4] [--nt 1000] [--T 4] [--narrow] [--exact]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.solvers.pde import FWIForward  # noqa: E402
from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize  # noqa: E402
from red_diffeq.utils.synthetic import make_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ns", type=int, default=4)
ap.add_argument("--nt", type=int, default=1000)
ap.add_argument("--T", type=int, default=4)
ap.add_argument("--narrow", action="store_true")
ap.add_argument("--exact", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
ctx = dict(n_grid=3000, nt=a.nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=3000, ns=a.ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
v = v_normalize(torch.from_numpy(make_model("curvefault", 500, 3000, batch=1))).to(dev)
plan = fwi._plan(500, 3000, dev)
plan.set_variant(wide_chunked=not a.narrow, adj_exact=a.exact)
plan.set_tuning(a.T, a.T, 1)
sz = plan.sizes(1)
dseis = torch.randn(1, a.ns, sz.nrec, plan.ng, device=dev)
coeffs, vstat = plan.coeffs(v, 0)
seis, hist = plan.forward(coeffs, 1, keep_history=True)
gA, gk, gb = plan.adjoint(coeffs, hist, dseis, 1)
torch.cuda.synchronize()
plan.status()
print("ok", float(gA.double().abs().sum()))
