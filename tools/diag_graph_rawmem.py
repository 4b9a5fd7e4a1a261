"""Diagnostic: tools/diag_graph_memset.py with every buffer the forward graph touches allocated by
hipMalloc directly (not torch's caching allocator) and filled / read with hipMemset / hipMemcpy on
the null stream; coeffs still come from the plan (copied into a hipMalloc buffer)."""
import ctypes, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "red-diffeq_amd"), ROOT]
from conftest import ctx_of, load_golden, vnorm        # noqa: E402
from test_gpu_fwi import make_fwi                       # noqa: E402
from red_diffeq import _hip                             # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
def hmalloc(nbytes):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) == 0
    return p
def hset(p, byte, nbytes):
    assert hip.hipMemset(p, ctypes.c_int(byte), ctypes.c_size_t(nbytes)) == 0
def hget(p, nfloats):
    a = np.empty(nfloats, np.float32)
    assert hip.hipMemcpy(a.ctypes.data_as(ctypes.c_void_p), p, ctypes.c_size_t(4 * nfloats), 2) == 0
    return a

z = load_golden(sys.argv[1] if len(sys.argv) > 1 else "fwd_wrap")
fwi = make_fwi(ctx_of(z))
v = torch.from_numpy(vnorm(z["v"])).to("cuda")
B = v.shape[0]
plan = fwi._plan(v.shape[2], v.shape[3], v.device)
plan.set_persistent(False)
sz = plan.sizes(B)
coeffs_t, _ = plan.coeffs(v, 0)
torch.cuda.synchronize()
nco = coeffs_t.numel()
coeffs = hmalloc(4 * nco)
assert hip.hipMemcpy(coeffs, ctypes.c_void_p(coeffs_t.data_ptr()), ctypes.c_size_t(4 * nco), 3) == 0
nseis = B * plan.ns * sz.nrec * plan.ng
seis = hmalloc(4 * nseis)
nh = int(sz.history) // 4
hist = hmalloc(4 * nh)
ring = hmalloc(int(sz.ring))
head = 2 * B * plan.ns * sz.Hp * sz.ld
ref = None
for graphs in (False, True):
    plan.set_graphs(graphs)
    for trial in range(4):
        hset(hist, 0xFF, 4 * nh)          # 0xFFFFFFFF = NaN
        hset(seis, 0xFF, 4 * nseis)
        hip.hipDeviceSynchronize()
        rc = plan.lib.rdq_fwi_forward(plan.handle, B, coeffs, seis, hist, ring, ctypes.c_void_p(0))
        hip.hipDeviceSynchronize()
        h = hget(hist, nh)
        s = hget(seis, nseis)
        if ref is None:
            ref = s
        print(json.dumps({"graphs": graphs, "trial": trial, "rc": rc,
                          "head_nonzero": int((h[:head] != 0).sum()), "head_nan": int(np.isnan(h[:head]).sum()),
                          "seis_nan": int(np.isnan(s).sum()),
                          "seis_eq_direct": bool(np.array_equal(s.view(np.int32), ref.view(np.int32)))}), flush=True)
