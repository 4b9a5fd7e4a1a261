"""Diagnostic: persistent adjoint (FMA / exact) vs chunked exact vs the oracle on one config."""
import sys
import numpy as np
import torch
sys.path.insert(0, "red-diffeq_amd"); sys.path.insert(0, ".")
from oracle import oracle as O
from red_diffeq.solvers.pde import FWIForward
from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
from red_diffeq.utils.synthetic import make_model

B, ns, nt = (int(x) for x in sys.argv[1:4])
dev = torch.device("cuda:0")
ctx = dict(n_grid=70, nt=nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
vn = ((make_model("curvevel", 70, 70, seed=5, batch=B) - 1500) / 3000 * 2 - 1).astype(np.float32)
v = torch.from_numpy(vn).to(dev)
plan = fwi._plan(70, 70, dev)
sz = plan.sizes(B)
rng = np.random.default_rng(1)
ds_np = rng.standard_normal((B, ns, sz.nrec, 70)).astype(np.float32)
ds = torch.from_numpy(ds_np).to(dev)
res = {}
for name, persist, exact in (("pt_fma", True, False), ("pt_exact", True, True), ("tb_exact", False, True)):
    plan.set_persistent(persist)
    plan.set_variant(adj_exact=exact)
    coeffs, vstat = plan.coeffs(v, 0)
    seis, hist = plan.forward(coeffs, B, keep_history=True)
    gA, gk, gb = plan.adjoint(coeffs, hist, ds, B)
    torch.cuda.synchronize()
    st = plan.debug_words()
    gAs = gA.view(B, ns, sz.Hp, sz.ld)[..., :sz.Wp].cpu().numpy().astype(np.float64).sum(1)
    res[name] = (gAs, gb.cpu().numpy().reshape(B, ns), gk.view(B, -1).sum(1).cpu().numpy())
    print(name, "status", st[0], "launch", plan.launch_info(B), flush=True)
    plan.status() if st[0] == 0 else None
    del hist
f = O.OracleFWI(ctx, B)
_, c = f.forward(vn, keep_history=True)
oA, oK, ob = f.adjoint(c, ds_np)
for name, (gA, gb, gk) in res.items():
    ra = np.linalg.norm(gA - oA) / np.linalg.norm(oA)
    rb = np.abs(gb - ob).max() / np.abs(ob).max()
    rk = np.abs(gk - oK).max() / np.abs(oK).max()
    bad = np.argwhere(np.abs(gA - oA) > 1e-3 * np.abs(oA).max())
    print(f"{name}: gA rel {ra:.2e} gb {rb:.2e} gk {rk:.2e} bad cells {len(bad)} first {bad[:5].tolist()}", flush=True)
