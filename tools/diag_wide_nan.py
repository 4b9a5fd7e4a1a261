"""Diagnostic: repeat the chunked forward + wide adjoint on a golden forward fixture with graphs on and
off and report, per output (seis, gA, gbeta, gk, dL/dv), whether a repeat matches the graphs-off
result bit for bit, and where the first differing cells are."""
import argparse, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "red-diffeq_amd"), ROOT]
from conftest import ctx_of, load_golden, vnorm        # noqa: E402
from test_gpu_fwi import _chunked_run, make_fwi         # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--name", default="fwd_wrap")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--Tw", type=str, default="5,6")
ap.add_argument("--T", type=int, default=4)
a = ap.parse_args()
z = load_golden(a.name)
ctx = ctx_of(z)
fwi = make_fwi(ctx)
vn = vnorm(z["v"])
v = torch.from_numpy(vn).to("cuda")
B = v.shape[0]
plan = fwi._plan(v.shape[2], v.shape[3], v.device)
sz = plan.sizes(B)
print(json.dumps({"Hp": sz.Hp, "Wp": sz.Wp, "ld": sz.ld, "B": B, "ns": plan.ns, "nt": plan.nt if hasattr(plan, "nt") else None}), flush=True)
rng = np.random.default_rng(3)
dseis = torch.from_numpy(rng.standard_normal((B, plan.ns, sz.nrec, plan.ng)).astype(np.float32)).cuda()
names = ("seis", "gA", "gbeta", "gk", "g")


def hist_head(T, Tw, graphs):
    """The forward's history slots 0 and 1 (P_{-1}, P_0: zeroed by the forward's first memset)."""
    plan.set_graphs(graphs)
    plan.set_persistent(False)
    plan.set_variant(wide_chunked=True)
    plan.set_tuning(T, T, 1)
    coeffs, _ = plan.coeffs(v, 0)
    junk = torch.full((64 << 20,), float("nan"), device="cuda")   # recycled memory holds NaN
    del junk
    seis, hist = plan.forward(coeffs, B, keep_history=True)
    h = hist.view(-1)[: 2 * sz.Hp * sz.ld * B * plan.ns]
    return float(torch.nan_to_num(h, nan=1e30).abs().max()), bool(torch.isfinite(seis).all())
for Tw in [int(x) for x in a.Tw.split(",")]:
    plan.set_graphs(False)
    ref = _chunked_run(plan, v, B, dseis, True, False, a.T, Tw=Tw)
    plan.set_graphs(True)
    for rep in range(a.reps):
        out = _chunked_run(plan, v, B, dseis, True, False, a.T, Tw=Tw)
        rec = {"Tw": Tw, "rep": rep}
        for n, x, y in zip(names, out, ref):
            eq = bool(np.array_equal(np.ascontiguousarray(x, np.float32).view(np.int32),
                                     np.ascontiguousarray(y, np.float32).view(np.int32)))
            rec[n] = eq
            if not eq:
                d = np.argwhere(np.ascontiguousarray(x, np.float32).view(np.int32)
                                != np.ascontiguousarray(y, np.float32).view(np.int32))
                rec[n + "_ndiff"] = int(len(d))
                rec[n + "_first"] = d[:6].tolist()
                rec[n + "_finite"] = bool(np.isfinite(x).all())
                if n == "gbeta":
                    rec["gbeta_ratio"] = (np.asarray(x, np.float64).ravel() / np.asarray(y, np.float64).ravel()).tolist()
        print(json.dumps(rec), flush=True)
for rep in range(3):
    print(json.dumps({"hist_head_rep": rep, "graphs_on": hist_head(a.T, 6, True), "graphs_off": hist_head(a.T, 6, False)}), flush=True)
