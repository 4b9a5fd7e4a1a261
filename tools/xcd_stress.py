"""Stress the persistent kernels' hand-offs: N asynchronous forward+adjoint pairs (fresh buffers
from the caching allocator each time, as in an inversion loop), then one status check.
python tools/xcd_stress.py [--pairs 40] [--no-xcd] [--no-graphs]"""
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
ap.add_argument("--pairs", type=int, default=40)
ap.add_argument("--ns", type=int, default=8)
ap.add_argument("--nt", type=int, default=1000)
ap.add_argument("--no-xcd", action="store_true")
ap.add_argument("--no-graphs", action="store_true")
ap.add_argument("--fwd-only", action="store_true")
ap.add_argument("--junk", action="store_true", help="interleave unrelated kernels writing scratch tensors")
a = ap.parse_args()
dev = torch.device("cuda:0")
ctx = dict(n_grid=70, nt=a.nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=a.ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
v = v_normalize(torch.from_numpy(make_model("flatvel", 70, 70, batch=1))).to(dev)
plan = fwi._plan(70, 70, dev)
plan.set_variant(xcd_local=not a.no_xcd)
if a.no_graphs:
    plan.set_graphs(False)
sz = plan.sizes(1)
dseis = torch.randn(1, a.ns, sz.nrec, plan.ng, device=dev)
for i in range(a.pairs):
    coeffs, vstat = plan.coeffs(v, 0)
    seis, hist = plan.forward(coeffs, 1, keep_history=True)
    if a.junk:
        t = torch.randn(int(sz.ring) // 4 + 12345, device=dev)
        t.mul_(2.0)
        del t
    if not a.fwd_only:
        plan.adjoint(coeffs, hist, dseis, 1)
    del hist
    if (i + 1) % 10 == 0:
        w = plan.debug_words()
        print(i, w, flush=True)
        if w[0]:
            plan.status() if False else None
            sys.exit(3)
