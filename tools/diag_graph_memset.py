"""Diagnostic: the chunked forward through the C ABI on fixed buffers whose history is pre-filled
with NaN: with graphs the first call captures and later calls replay; the history's first two
slots (P_{-1}, P_0) must read zero afterwards (the forward's memset).  With / without a device
synchronisation between the NaN fill and the call."""
import ctypes, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "red-diffeq_amd"), ROOT]
from conftest import ctx_of, load_golden, vnorm        # noqa: E402
from test_gpu_fwi import make_fwi                       # noqa: E402
from red_diffeq import _hip                             # noqa: E402

z = load_golden(sys.argv[1] if len(sys.argv) > 1 else "fwd_wrap")
fwi = make_fwi(ctx_of(z))
v = torch.from_numpy(vnorm(z["v"])).to("cuda")
B = v.shape[0]
plan = fwi._plan(v.shape[2], v.shape[3], v.device)
plan.set_persistent(False)
sz = plan.sizes(B)
coeffs, _ = plan.coeffs(v, 0)
seis = torch.empty(B, plan.ns, sz.nrec, plan.ng, device="cuda")
hist = torch.empty(int(sz.history) // 4, device="cuda")
ring = torch.empty(int(sz.ring) // 4, device="cuda")
head = 2 * B * plan.ns * sz.Hp * sz.ld
st = torch.cuda.current_stream().cuda_stream
print(json.dumps({"stream": st, "head": head, "hist_floats": hist.numel()}), flush=True)
for graphs in (True, False):
    plan.set_graphs(graphs)
    for sync in (False, True):
        for trial in range(3):
            hist.fill_(float("nan"))
            seis.fill_(float("nan"))
            if sync:
                torch.cuda.synchronize()
            rc = plan.lib.rdq_fwi_forward(plan.handle, B, _hip.ptr(coeffs), _hip.ptr(seis), _hip.ptr(hist),
                                          _hip.ptr(ring), ctypes.c_void_p(st))
            torch.cuda.synchronize()
            h = hist[:head]
            lvl = head // 2
            s0 = int((hist[:lvl] != 0).sum()); s1 = int((hist[lvl:head] != 0).sum())
            same = [bool(torch.equal(hist[j * lvl:(j + 1) * lvl], hist[0:lvl])) for j in range(2, 8)] if s0 else []
            print(json.dumps({"graphs": graphs, "sync": sync, "trial": trial, "rc": rc,
                              "head_nan": int(torch.isnan(h).sum()), "head_nonzero": int((h != 0).sum()),
                              "seis_nan": int(torch.isnan(seis).sum()),
                              "slot0_nonzero": s0, "slot1_nonzero": s1, "slot0_equals_slot": same,
                              "seis_nan_at": torch.nonzero(torch.isnan(seis))[:4].tolist()}), flush=True)
