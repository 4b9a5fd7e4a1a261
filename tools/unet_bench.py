"""Time the HIP U-Net forward (csrc/unet.hip) at the reference inversion configuration
(dim 64, mults 1,2,4,8, 1 channel, 72x72; red_diffeq/models/diffusion.py:220-301) against the
PyTorch-ROCm eager forward of the same weights (tests/unet_torch_ref.py), and report conv
FLOP/s against the fp32 matrix-core peak.
python tools/unet_bench.py [--B 1 4] [--reps 20]"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from red_diffeq.models.diffusion import Unet  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X dense fp32 matrix (MI355X_MICROARCH.md)


def conv_flops(net, x, t):
    """2 x MACs of every convolution of one HIP forward (counted at the ops.conv2d boundary)."""
    from red_diffeq.models import unet_ops as ops
    tot = [0]
    orig = ops.conv2d

    def counting(x, conv, x2=None, mode=ops.PLAIN, residual=None):
        y = orig(x, conv, x2=x2, mode=mode, residual=residual)
        cout, cin, kh, kw = conv.weight.shape
        tot[0] += 2 * y.shape[0] * y.shape[2] * y.shape[3] * cout * cin * kh * kw
        return y

    ops.conv2d = counting
    os.environ["RDQ_NO_UNET_GRAPH"] = "1"          # one eager forward (a graph capture runs it twice)
    try:
        with torch.no_grad():
            net(x, t)
    finally:
        ops.conv2d = orig
        del os.environ["RDQ_NO_UNET_GRAPH"]
    return tot[0]


def conv_shapes(net, x, t):
    """(x shape, x2 channels, conv, mode, residual?) of every convolution of one forward."""
    from red_diffeq.models import unet_ops as ops
    calls = []
    orig = ops.conv2d

    def rec(x, conv, x2=None, mode=ops.PLAIN, residual=None):
        calls.append((tuple(x.shape), 0 if x2 is None else x2.shape[1], conv, mode, residual is not None))
        return orig(x, conv, x2=x2, mode=mode, residual=residual)

    ops.conv2d = rec
    os.environ["RDQ_NO_UNET_GRAPH"] = "1"
    try:
        with torch.no_grad():
            net(x, t)
    finally:
        ops.conv2d = orig
        del os.environ["RDQ_NO_UNET_GRAPH"]
    return calls


def per_conv(net, x, t, reps):
    from red_diffeq.models import unet_ops as ops
    rows = []
    for xs, c2, conv, mode, has_res in conv_shapes(net, x, t):
        xa = torch.randn(xs, device="cuda")
        x2 = torch.randn(xs[0], c2, xs[2], xs[3], device="cuda") if c2 else None
        y = ops.conv2d(xa, conv, x2=x2, mode=mode)
        res = torch.randn_like(y) if has_res else None
        ms = time_fn(lambda: ops.conv2d(xa, conv, x2=x2, mode=mode, residual=res), reps)
        cout, cin, kh, kw = conv.weight.shape
        fl = 2 * y.shape[0] * y.shape[2] * y.shape[3] * cout * cin * kh * kw
        rows.append({"x": list(xs), "cin2": c2, "cout": cout, "k": kh, "mode": mode, "HW": y.shape[2],
                     "us": round(ms * 1e3, 2), "tflops": round(fl / ms / 1e9, 2)})
    rows.sort(key=lambda r: -r["us"])
    tot = sum(r["us"] for r in rows)
    print(json.dumps({"convs": len(rows), "sum_us": round(tot, 1)}))
    for r in rows:
        print(json.dumps(r))


def time_fn(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--H", type=int, default=72)
    ap.add_argument("--per-conv", action="store_true")
    a = ap.parse_args()
    import unet_torch_ref as R
    torch.manual_seed(0)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
    for B in a.B:
        x = torch.randn(B, 1, a.H, a.H, device="cuda")
        t = torch.randint(0, 1000, (B,), device="cuda")
        if a.per_conv:
            per_conv(net, x, t, a.reps)
            continue
        fl = conv_flops(net, x, t)
        with torch.no_grad():
            hip_ms = time_fn(lambda: net(x, t), a.reps)             # default path (graph replay if small)
            os.environ["RDQ_NO_UNET_GRAPH"] = "1"
            eager_ms = time_fn(lambda: net(x, t), a.reps)
            del os.environ["RDQ_NO_UNET_GRAPH"]
            ref_ms = time_fn(lambda: R.unet_forward(net, x, t), a.reps)
            d = (net(x, t) - R.unet_forward(net, x, t)).abs().max().item()
        out = {"B": B, "H": a.H, "conv_gflop": round(fl / 1e9, 3), "hip_ms": round(hip_ms, 3),
               "hip_eager_launch_ms": round(eager_ms, 3),
               "torch_eager_ms": round(ref_ms, 3), "hip_conv_tflops": round(fl / hip_ms / 1e9, 2),
               "mfma_frac_of_fp32_peak": round(fl / hip_ms / 1e9 / FP32_MFMA_PEAK_TFLOPS, 4),
               "max_abs_diff_vs_torch": d}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
