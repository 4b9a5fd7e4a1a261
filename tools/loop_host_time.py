"""Is the notebook-configuration RED loop host-bound?  The main stream is held by a long
torch.cuda._sleep, so every launch of `steps` iterations is only enqueued; the time the host takes to
reach the loop's first device -> host copy (the final history read) is its enqueue time per
iteration, set against the untimed-sleep wall time per iteration.
python tools/loop_host_time.py [steps] -> one JSON line per regulariser."""
import json
import warnings
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "red-diffeq_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
import notebook_floor as nf  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
marks = []
orig_cpu = torch.Tensor.cpu


def cpu(self, *a, **k):
    marks.append(time.perf_counter())
    return orig_cpu(self, *a, **k)


def calib():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(100_000_000)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 100_000_000     # ms per cycle


warnings.simplefilter("always")
ms_per_cycle = calib()
for reg in ("diffusion", "none"):
    run = nf.make_loop(dev, reg)
    run(3)
    torch.cuda.synchronize()
    hold_ms = 20.0 * steps + 200.0
    torch.cuda._sleep(int(hold_ms / ms_per_cycle))
    marks.clear()
    torch.Tensor.cpu = cpu
    if os.environ.get("SYNC_DEBUG"):
        torch.cuda.set_sync_debug_mode("warn")     # every synchronising call: a warning + its caller
    t0 = time.perf_counter()
    run(steps, sync=False)
    torch.cuda.set_sync_debug_mode(0)
    torch.Tensor.cpu = orig_cpu
    t_enq = (marks[0] - t0) * 1e3 if marks else float("nan")
    torch.cuda.synchronize()
    print(json.dumps({"reg": reg, "steps": steps, "hold_ms": hold_ms,
                      "host_enqueue_ms_per_iter": round(t_enq / steps, 3),
                      "enqueue_blocked": t_enq > hold_ms * 0.9,
                      "cpu_calls_ms": [round((m - t0) * 1e3, 2) for m in marks]}), flush=True)
