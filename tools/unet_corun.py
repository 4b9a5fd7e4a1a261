"""Does the B = 1 U-Net slow down beside the persistent FWI kernels?  The RED loop runs the U-Net on
a side stream next to the forward / adjoint (5 OpenFWI shots: 5 slices on 5 XCDs, 28 of their 32
CUs each).  Times one U-Net forward (graph replay, static I/O) alone, then started together with a
persistent forward, then together with an adjoint, each on its own stream with HIP events.
RDQ_CORUN_NULL=1: a graph of 114 one-workgroup kernels instead of the U-Net (same launch count, no
work): separates dispatch interference from the U-Net's compute / memory traffic.
python tools/unet_corun.py [ns] -> one JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "red-diffeq_amd")]
from red_diffeq.models.diffusion import Unet  # noqa: E402
from red_diffeq.solvers.pde import FWIForward  # noqa: E402
from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize  # noqa: E402
from red_diffeq.utils.synthetic import make_model  # noqa: E402

ns = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
torch.set_grad_enabled(False)          # graph_io captures the no-grad forward
torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(dev).eval()
xs, ts = net.graph_io((1, 1, 72, 72), dev)
xs.copy_(torch.randn(1, 1, 72, 72, device=dev))
ts.copy_(torch.randint(0, 1000, (1,), device=dev))
ctx = dict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
v = v_normalize(torch.from_numpy(make_model("curvefault", 70, 70, batch=1))).to(dev)
plan = fwi._plan(70, 70, dev)
sz = plan.sizes(1)
dseis = torch.randn(1, ns, sz.nrec, plan.ng, device=dev)
side = torch.cuda.Stream(device=dev)
if os.environ.get("RDQ_CORUN_NULL"):
    tiny = torch.zeros(256, device=dev)
    g_null = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        tiny.add_(1.0)
        side.synchronize()
        with torch.cuda.graph(g_null, stream=side):
            for _ in range(114):
                tiny.add_(1.0)

    class _Null:
        @staticmethod
        def replay_static(*_):
            g_null.replay()
    net = _Null()
main = torch.cuda.current_stream(dev)


def ev():
    return torch.cuda.Event(enable_timing=True)


def unet_alone():
    torch.cuda.synchronize()
    e0, e1 = ev(), ev()
    with torch.cuda.stream(side):
        e0.record()
        net.replay_static(xs, ts)
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def corun(phase):
    coeffs, _ = plan.coeffs(v, 0)
    if phase == "adjoint":
        _, hist = plan.forward(coeffs, 1, keep_history=True)
    torch.cuda.synchronize()
    e0, e1, f0, f1 = ev(), ev(), ev(), ev()
    f0.record()
    with torch.cuda.stream(side):
        side.wait_stream(main)
        e0.record()
        net.replay_static(xs, ts)
        e1.record()
    if phase == "forward":
        plan.forward(coeffs, 1, keep_history=True)
    else:
        plan.adjoint(coeffs, hist, dseis, 1)
    f1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), f0.elapsed_time(f1)


def fwi_alone(phase):
    coeffs, _ = plan.coeffs(v, 0)
    _, hist = plan.forward(coeffs, 1, keep_history=True)
    torch.cuda.synchronize()
    f0, f1 = ev(), ev()
    f0.record()
    if phase == "forward":
        plan.forward(coeffs, 1, keep_history=True)
    else:
        plan.adjoint(coeffs, hist, dseis, 1)
    f1.record()
    torch.cuda.synchronize()
    return f0.elapsed_time(f1)


with torch.no_grad():
    for _ in range(3):
        unet_alone()
        corun("forward")
        corun("adjoint")
    med = lambda xs_: sorted(xs_)[len(xs_) // 2]   # noqa: E731
    out = {"ns": ns, "null": bool(os.environ.get("RDQ_CORUN_NULL")), "info": plan.launch_info(1),
           "unet_alone_ms": med([unet_alone() for _ in range(7)])}
    for ph in ("forward", "adjoint"):
        r = [corun(ph) for _ in range(7)]
        out[f"unet_beside_{ph}_ms"] = med([a for a, _ in r])
        out[f"{ph}_with_unet_ms"] = med([b for _, b in r])
        out[f"{ph}_alone_ms"] = med([fwi_alone(ph) for _ in range(5)])
    plan.status()
print(json.dumps({k: (round(x, 3) if isinstance(x, float) else x) for k, x in out.items()}), flush=True)
