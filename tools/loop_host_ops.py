"""Host (CPU) time per operator inside the RED-DiffEq loop (notebook configuration), from
torch.profiler: which host calls keep the next iteration's forward from being enqueued early."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
import bench  # noqa: E402

dev = torch.device("cuda")
a = argparse.Namespace(nt=1000, steps=1, warmup=1)
bench.red_loop_wallclock(dev, a, ns=5, family="curvefault")     # warm everything up
a.steps = 8
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
    print("ms/iter", bench.red_loop_wallclock(dev, a, ns=5, family="curvefault"), flush=True)
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30, max_name_column_width=60))
