"""Gradient of a wrap-geometry fixture (region larger than the grid) vs the oracle under each
adjoint / forward kernel choice: isolates which kernel disagrees.  Usage: python tools/diag_wrap.py [name]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "red-diffeq_amd"), os.path.join(ROOT, "tests")]
from conftest import ctx_of, load_golden, vnorm   # noqa: E402
from oracle import oracle as O                      # noqa: E402
from test_gpu_fwi import make_fwi                   # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "fwd_wrap"
z = load_golden(name)
dev = torch.device("cuda:0")
v0 = vnorm(z["v"])
f = O.OracleFWI(ctx_of(z), v0.shape[0])
seis_o, c = f.forward(v0, keep_history=True)
ds = np.sign(np.random.default_rng(3).standard_normal(seis_o.shape)).astype(np.float32)
go = f.finalize(c, *f.adjoint(c, ds))
for label, kw in [("default", {}), ("adj_exact", dict(adj_exact=True)), ("chunked", dict(persist=False)),
                  ("fwd_chunked_only", dict(fwd_chunked=True)), ("T2", dict(T=2)), ("T1", dict(T=1))]:
    fwi = make_fwi(ctx_of(z))
    v = torch.from_numpy(v0).to(dev).requires_grad_(True)
    plan = fwi._plan(v.shape[2], v.shape[3], dev)
    if "T" in kw:
        plan.set_tuning(kw["T"], kw["T"], 1)
    plan.set_variant(adj_exact=kw.get("adj_exact", False))
    if kw.get("persist") is False:
        plan.set_persistent(False)
    seis = fwi(v)
    if kw.get("fwd_chunked"):
        pass
    seis.backward(torch.from_numpy(ds).to(dev))
    plan.status()
    g = v.grad.cpu().numpy()
    err = float(np.linalg.norm(g - go) / np.linalg.norm(go))
    d = np.abs(g - go)[0, 0]
    iz, ix = np.unravel_index(np.argmax(d), d.shape)
    print(json.dumps({"case": label, "info": plan.launch_info(1), "rel_l2": err,
                      "worst_cell": [int(iz), int(ix)], "seis_bits_equal":
                      bool(np.array_equal(seis.detach().cpu().numpy().view(np.int32), seis_o.astype(np.float32).view(np.int32)))}))
    rowerr = np.abs(g - go)[0, 0].max(axis=1) / (np.abs(go).max() + 1e-30)
    print("  row max err:", np.array2string(rowerr, precision=2, max_line_width=200))
