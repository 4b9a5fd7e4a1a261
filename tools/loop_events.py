"""Device and host timeline of the notebook-configuration RED loop without a profiler (rocprofv3's
kernel trace serialises the queues): HIP events on the issuing stream and host clocks at the
regulariser (side stream), the data term (after the forward), Adam, and each iteration's end.
python tools/loop_events.py [steps] -> per-iteration JSON lines (ms from the iteration's first event):
{tag: [device ms, host ms]}, ">" at entry, "<" at exit."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "red-diffeq_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
import notebook_floor as nf  # noqa: E402
from red_diffeq.core import fused, losses  # noqa: E402
from red_diffeq.solvers import pde  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reg = sys.argv[2] if len(sys.argv) > 2 else "diffusion"
dev = torch.device("cuda:0")
log = []


def mark(tag):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    log.append((tag, e, time.perf_counter()))


def wrap(cls, name, tag):
    f = getattr(cls, name)

    def g(*a, **k):
        mark(tag + ">")
        r = f(*a, **k)
        mark(tag + "<")
        return r
    setattr(cls, name, g)


wrap(losses.LossCalculator, "regularization_loss", "reg")
wrap(losses.LossCalculator, "observation_loss", "obs")
wrap(pde.FWIForward, "forward", "fwd")
wrap(fused.FusedAdamClamp, "step", "adam")
run = nf.make_loop(dev, None if reg == "none" else reg)
run(3)
log.clear()
run(steps)
torch.cuda.synchronize()
first = "reg>" if reg == "diffusion" else "fwd>"
it_starts = [i for i, (t, _, _) in enumerate(log) if t == first]
for a, b in zip(it_starts, it_starts[1:] + [len(log)]):
    e0, h0 = log[a][1], log[a][2]
    row = {t: [round(e0.elapsed_time(e), 3), round((h - h0) * 1e3, 3)] for t, e, h in log[a:b]}
    if b < len(log):
        row["next"] = [round(e0.elapsed_time(log[b][1]), 3), round((log[b][2] - h0) * 1e3, 3)]
    print(json.dumps(row), flush=True)
