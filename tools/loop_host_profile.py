"""Host-side cost of one RED-DiffEq iteration (the reference notebook's configuration: CurveFault
70x70, ns = 5, B = 1): wallclock per iteration vs the device time the iteration's stream work takes,
and a cProfile of the host (is the loop host-bound?)."""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ns", type=int, default=5)
ap.add_argument("--iters", type=int, default=30)
a = ap.parse_args()
dev = torch.device("cuda")
args = argparse.Namespace(nt=1000, steps=a.iters, warmup=3)
print("wallclock ms/iter", bench.red_loop_wallclock(dev, args, ns=a.ns, family="curvefault"), flush=True)
args.steps = 10
pr = cProfile.Profile()
pr.enable()
ms = bench.red_loop_wallclock(dev, args, ns=a.ns, family="curvefault")
pr.disable()
print("under cProfile ms/iter", ms, flush=True)
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
