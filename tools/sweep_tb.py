"""Time the forward / adjoint time loops for every temporal-blocking depth (steps per launch).
python tools/sweep_tb.py [--ns 8] [--B 1]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.solvers.pde import FWIForward  # noqa: E402
from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize  # noqa: E402
from red_diffeq.utils.synthetic import make_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ns", type=int, default=8)
ap.add_argument("--B", type=int, default=1)
ap.add_argument("--nt", type=int, default=1000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--only", type=int, default=0, help="run a single blocking depth")
ap.add_argument("--chunked", action="store_true", help="also time the chunked (launch per T steps) kernels")
ap.add_argument("--profile", action="store_true", help="phase counters of the persistent kernels")
ap.add_argument("--mode", type=int, default=1, help="persistent mode: 1 auto, 12 / 8 region height")
ap.add_argument("--rw", default=None, help="rows per wave of the 96-row kernels, 'fwd,adj' (e.g. 12,12)")
ap.add_argument("--delay", default=None, help="pre-sweep delays of the persistent kernels, 'fwd,adj' ticks")
a = ap.parse_args()
dev = torch.device("cuda:0")
ctx = dict(n_grid=70, nt=a.nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=a.ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
v = v_normalize(torch.from_numpy(make_model("flatvel", 70, 70, batch=a.B))).to(dev)
plan = fwi._plan(70, 70, dev)
if a.rw:
    plan.set_rows_per_wave(*[int(x) for x in a.rw.split(",")])
if a.delay:
    plan.set_sweep_delay(*[int(x) for x in a.delay.split(",")])
sz = plan.sizes(a.B)
dseis = torch.randn(a.B, a.ns, sz.nrec, plan.ng, device=dev)
res = []
# (T, persistent)
cfgs = [(a.only, a.mode)] if a.only else [(2, a.mode), (3, a.mode), (4, a.mode)]
if a.chunked:
    cfgs += [(T, 0) for T in (2, 3, 4)]
for T, G in cfgs:
    plan.set_tuning(T, T, 1)
    plan.set_persistent(G)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fw, ad = [], []
    for i in range(a.reps + 1):
        coeffs, vstat = plan.coeffs(v, 0)
        ev[0].record()
        seis, hist = plan.forward(coeffs, a.B, keep_history=True)
        ev[1].record()
        plan.adjoint(coeffs, hist, dseis, a.B)
        ev[2].record()
        torch.cuda.synchronize()
        if i:
            fw.append(ev[0].elapsed_time(ev[1]))
            ad.append(ev[1].elapsed_time(ev[2]))
        del hist
    plan.status()
    fw, ad = sorted(fw)[len(fw) // 2], sorted(ad)[len(ad) // 2]
    res.append({"T": T, "persistent": G, "mode": a.mode, "rw": a.rw, "delay": a.delay, "ns": a.ns,
                "fwd_launches": plan.launch_info(a.B)["fwd_launches"], "fwd_ms": round(fw, 3), "adj_ms": round(ad, 3),
                "shot_ts_per_s": round(a.ns * a.nt * a.B / ((fw + ad) * 1e-3))})
    if a.profile and G:
        plan.set_profile(1)
        coeffs, vstat = plan.coeffs(v, 0)
        seis, hist = plan.forward(coeffs, a.B, keep_history=True)
        plan.adjoint(coeffs, hist, dseis, a.B)
        prof = plan.read_profile()
        import numpy as np
        for name, adj in (("fwd", 0), ("adj", 1)):
            wv = plan.profile_waves(adj)
            live = wv[wv.sum(1) > 0]
            ids = np.nonzero(wv.sum(1) > 0)[0]
            tot = live.sum(1)
            st = live[:, 1]
            slow = ids[np.argsort(st)[-6:]]
            prof[name]["steps_us_min_med_max"] = [round(float(np.min(st)), 1), round(float(np.median(st)), 1),
                                                  round(float(np.max(st)), 1)]
            prof[name]["total_us_min_max"] = [round(float(tot.min()), 1), round(float(tot.max()), 1)]
            prof[name]["slowest_block_wave"] = [(int(i) // 16, int(i) % 16) for i in slow]
            # per block: hand-off wait summed over its waves; the critical-path blocks wait least
            blk = {}
            for i, v in zip(ids, live[:, 0]):
                blk.setdefault(int(i) // 16, []).append(v)
            bw = sorted((float(np.mean(v)), b) for b, v in blk.items())
            prof[name]["least_waiting_blocks"] = [(b, round(v, 1)) for v, b in bw[:8]]
            prof[name]["most_waiting_blocks"] = [(b, round(v, 1)) for v, b in bw[-4:]]
            # steps by wave index
            byw = {}
            for i, v in zip(ids, st):
                byw.setdefault(int(i) % 16, []).append(v)
            prof[name]["steps_us_by_wave"] = {k: round(float(np.mean(v)), 1) for k, v in sorted(byw.items())}
        plan.set_profile(0)
        del hist
        res[-1]["profile_us_per_wave"] = {k: {kk: (round(vv, 1) if isinstance(vv, float) else vv)
                                              for kk, vv in d.items()} for k, d in prof.items()}
    print(json.dumps(res[-1]), flush=True)
