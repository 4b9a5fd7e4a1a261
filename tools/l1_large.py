"""L1 misfit at configs[4]'s per-rank size (1 model x 16 shots x 1000 records x 3000 receivers) and at the
B = 25 yaml's (25 models x 5 x 1000 x 70): device time per call and the loss against a float64 torch sum.
python tools/l1_large.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq import ops  # noqa: E402,F401

for shape in ((1, 16, 1000, 3000), (25, 5, 1000, 70)):
    g = torch.Generator(device="cuda").manual_seed(0)
    pred = torch.randn(shape, device="cuda", generator=g)
    y = torch.randn(shape, device="cuda", generator=g)
    for _ in range(3):
        loss, nobs = torch.ops.red_diffeq.l1_misfit(pred, y, None)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        loss, nobs = torch.ops.red_diffeq.l1_misfit(pred, y, None)
    e1.record()
    torch.cuda.synchronize()
    ref = (y.double() - pred.double()).abs().flatten(1).mean(1)
    print(json.dumps({"shape": shape, "us_per_call": round(e0.elapsed_time(e1) * 1e3 / 20, 1),
                      "max_rel_vs_fp64": float(((loss.double() - ref).abs() / ref).max())}), flush=True)
