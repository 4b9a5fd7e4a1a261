"""Interleaved A/B of a U-Net kernel option (rdq_unet_set_option) on the dim-64 72 x 72 U-Net forward,
replayed from its captured graph with static I/O (the RED loop's path): for each round, each value is
set, the graph recaptured (the option generation is part of the cache key) and timed.
python tools/unet_opt_ab.py OPTION V1 V2 [...] [--B B] [--rounds R] [--reps N]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq import _hip  # noqa: E402
from red_diffeq.models.diffusion import Unet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("option", type=int)
ap.add_argument("values", type=int, nargs="+")
ap.add_argument("--B", type=int, default=1)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=200)
a = ap.parse_args()
torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
x = torch.randn(a.B, 1, 72, 72, device="cuda")
t = torch.randint(0, 1000, (a.B,), device="cuda")
lib = _hip.lib()
res = {v: [] for v in a.values}
outs = {}
with torch.no_grad():
    for r in range(a.rounds):
        for v in a.values:
            old = lib.rdq_unet_set_option(a.option, v)
            try:
                xs, ts = net.graph_io(x.shape, x.device)
                xs.copy_(x)
                ts.copy_(t)
                for _ in range(5):
                    y = net.replay_static(xs, ts)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    net.replay_static(xs, ts)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / a.reps)
                outs[v] = y.clone()
            finally:
                lib.rdq_unet_set_option(a.option, old)
ref = outs[a.values[0]]
for v in a.values:
    d = float((outs[v] - ref).abs().max() / ref.abs().max())
    print(json.dumps({"option": a.option, "value": v, "B": a.B, "ms": [round(m, 4) for m in res[v]],
                      "best_ms": round(min(res[v]), 4), "max_rel_diff_vs_first": d}), flush=True)
