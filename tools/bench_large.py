"""configs[4] (Marmousi-scale) FWI propagator timing on one MI355X: a 500 x 3000 synthetic model
(740 x 3240 padded, Npad = 2,397,600), `--ns` shots per GPU (16 = 128 shots sharded 8-way), ng = nx
receivers, nt = 1000, store-all history (16 shots: 155 GB of HBM).  One launch of this size does not
fit resident on the chip, so the chunked temporal-blocked kernels (k_fwd_tw / k_adj_tw; --narrow:
k_fwd_tb / k_adj_tb) run it.

Prints one JSON line per blocking depth: forward / adjoint ms, shot-timesteps/s, algorithmic GB/s
(12·Npad B per forward shot-step, 16·Npad B per adjoint shot-step).
python tools/bench_large.py [--ns 16] [--nz 500] [--nx 3000] [--nt 1000] [--reps 2]"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.solvers.pde import FWIForward  # noqa: E402
from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize  # noqa: E402
from red_diffeq.utils.synthetic import make_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ns", type=int, default=16)
ap.add_argument("--nz", type=int, default=500)
ap.add_argument("--nx", type=int, default=3000)
ap.add_argument("--nt", type=int, default=1000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--T", type=str, default="2,3,4", help="blocking depths to time")
ap.add_argument("--narrow", action="store_true", help="64-column chunked regions (round-3 layout)")
ap.add_argument("--exact", action="store_true", help="exact-order adjoint (RDQ_VARIANT_ADJ_EXACT)")
ap.add_argument("--chunked-adj-fma", action="store_true", help="contracted wide chunked adjoint (RDQ_VARIANT_CHUNKED_ADJ_FMA)")
ap.add_argument("--Tw", type=int, default=0, help="wide chunked adjoint depth (rdq_fwi_set_wide_adj_steps; 0 = auto)")
ap.add_argument("--spw", type=int, default=0, help="wide adjoint shots per workgroup (0: the plan's default)")
ap.add_argument("--fspw", type=int, default=0, help="wide forward shots per workgroup (0: the plan's default)")
ap.add_argument("--fTw", type=int, default=0, help="wide forward depth (0: the --T depth)")
ap.add_argument("--chains", type=int, default=0, help="concurrent shot-group launch chains")
ap.add_argument("--no-gen", action="store_true",
                help="chunked forward loads the K3 coefficient fields instead of regenerating them (the default)")
ap.add_argument("--phase", action="store_true",
                help="timing-only builds (RDQ_HIP_LIB) exporting rdq_exp_adj_phase: per-workgroup phase split of the "
                     "wide adjoint (launch start -> step 0's exchange, steps, epilogue), mean us per workgroup")
a = ap.parse_args()
dev = torch.device("cuda:0")
ctx = dict(n_grid=a.nx, nt=a.nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=a.nx, ns=a.ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
v = v_normalize(torch.from_numpy(make_model("curvefault", a.nz, a.nx, batch=1))).to(dev)
plan = fwi._plan(a.nz, a.nx, dev)
plan.set_variant(fwd_gen_coeffs=not a.no_gen, wide_chunked=not a.narrow, adj_exact=a.exact,
                 chunked_adj_fma=a.chunked_adj_fma)
plan.set_wide_adj_steps(a.Tw)
if a.spw:
    plan.set_wide_adj_shots(a.spw)
if a.fspw:
    plan.set_wide_fwd_shots(a.fspw)
plan.set_wide_fwd_steps(a.fTw)
sz = plan.sizes(1)
npad = sz.Hp * sz.Wp
dseis = torch.randn(1, a.ns, sz.nrec, plan.ng, device=dev)
print(json.dumps({"grid": [a.nz, a.nx], "padded": [sz.Hp, sz.Wp], "ld": sz.ld, "ns": a.ns, "nt": a.nt,
                  "history_GB": round(sz.history / 1e9, 2), "launch": plan.launch_info(1)}), flush=True)
for T in [int(t) for t in a.T.split(",")]:
    plan.set_tuning(T, T, a.chains)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fw, ad = [], []
    t0 = time.time()
    for i in range(a.reps + 1):
        coeffs, vstat = plan.coeffs(v, 0)
        ev[0].record()
        seis, hist = plan.forward(coeffs, 1, keep_history=True)
        ev[1].record()
        if a.phase and i == a.reps:
            torch.cuda.synchronize()
            ph = (ctypes.c_uint64 * 8)()
            plan.lib.rdq_exp_adj_phase(ph)          # read-and-reset
        plan.adjoint(coeffs, hist, dseis, 1)
        ev[2].record()
        torch.cuda.synchronize()
        if a.phase and i == a.reps:
            plan.lib.rdq_exp_adj_phase(ph)
            n = max(1, ph[3])
            print(json.dumps({"adj_phase_us_per_wg": {"start_to_step0_exchange": round(ph[0] / n / 100, 3),
                                                      "steps_after": round(ph[1] / n / 100, 3),
                                                      "epilogue": round(ph[2] / n / 100, 3)},
                              "workgroups": n}), flush=True)
        del hist
        if i:
            fw.append(ev[0].elapsed_time(ev[1]))
            ad.append(ev[1].elapsed_time(ev[2]))
    plan.status()
    f, d = min(fw), min(ad)
    shot_steps = a.ns * a.nt
    print(json.dumps({"T": T, "fwd_gen": not a.no_gen, "wide": not a.narrow, "exact": a.exact, "chunked_adj_fma": a.chunked_adj_fma, "Tw": a.Tw, "spw": a.spw, "fspw": a.fspw, "fTw": a.fTw, "chains": a.chains, "fwd_ms": round(f, 2), "adj_ms": round(d, 2),
                      "shot_ts_per_s": round(shot_steps / ((f + d) / 1e3)),
                      "fwd_GBps_alg": round(12 * npad * shot_steps / f / 1e6, 1),
                      "adj_GBps_alg": round(16 * npad * shot_steps / d / 1e6, 1),
                      "fwd_adj_frac_of_8TBps": round(28 * npad * shot_steps / (f + d) / 1e6 / 8000, 4),
                      "wall_s": round(time.time() - t0, 1)}), flush=True)
