"""Diagnostic: the dot-product test's inputs, full gradient per adjoint variant vs the oracle."""
import sys
import numpy as np
import torch
sys.path.insert(0, "red-diffeq_amd"); sys.path.insert(0, ".")
from oracle import oracle as O
from red_diffeq.solvers.pde import FWIForward
from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
from red_diffeq.utils.synthetic import make_model

dev = torch.device("cuda:0")
ctx = dict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=8)
torch.manual_seed(0)
v = torch.from_numpy(((make_model("curvevel", 70, 70, seed=5, batch=2) - 1500) / 3000 * 2 - 1).astype(np.float32)).to(dev).double()
v = v + 0.02 * torch.rand_like(v)
v[:, 0, 30, 40] = v.amin(dim=(1, 2, 3)) - 0.05
v = v.float()
vn = v.cpu().numpy()
f = O.OracleFWI(ctx, 2)
s_ref, c = f.forward(vn, keep_history=True)
w = np.random.default_rng(2).standard_normal(s_ref.shape).astype(np.float32)
oA, oK, ob = f.adjoint(c, w)
go = f.finalize(c, oA, oK, ob)
for exact in (True, False):
    for persist in (True, False):
        fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
        plan = fwi._plan(70, 70, dev)
        plan.set_variant(adj_exact=exact)
        plan.set_persistent(persist)
        vv = v.clone().requires_grad_(True)
        seis = fwi(vv)
        (seis * torch.from_numpy(w).to(dev)).sum().backward()
        fwi.check()
        g = vv.grad.cpu().numpy()
        rel = np.linalg.norm(g - go) / np.linalg.norm(go)
        i = np.unravel_index(np.argmax(np.abs(g - go)), g.shape)
        print(f"exact={exact} persist={persist}: grad rel {rel:.2e}, worst {i} got {g[i]:.4e} ref {go[i]:.4e}", flush=True)
