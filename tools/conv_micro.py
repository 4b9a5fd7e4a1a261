"""Per-shape timing of the U-Net's convolutions (dim 64, 72x72): each shape's op captured back to
back in a hipGraph, replayed, device time per call and TFLOP/s against the fp32 matrix peak, or with
--bf16 (the configs[4] batch: --B 344) against the bf16 dense peak.
python tools/conv_micro.py [--only NAME] [--reps R] [--B B ...] [--bf16] [--inner N] [--f32-min-tiles T ...]
(--f32-min-tiles: rdq_unet_set_option(RDQ_UNET_OPT_CONV3F_MIN_TILES) values to compare; 0 = per-tap only)"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq import _hip, ops  # noqa: E402

# name: (cin1, cin2, cout, k, H, mode)
SHAPES = {
    "l72_3x3_64_64": (64, 0, 64, 3, 72, 0),
    "l72_3x3_128_64": (64, 64, 64, 3, 72, 0),
    "l72_1x1_64_384": (64, 0, 384, 1, 72, 0),
    "l72_up_128_64": (128, 0, 64, 3, 72, 1),
    "l36_3x3_64_64": (64, 0, 64, 3, 36, 0),
    "l18_3x3_128_128": (128, 0, 128, 3, 18, 0),
    "l9_3x3_256_256": (256, 0, 256, 3, 9, 0),
    "l9_3x3_512_512": (512, 0, 512, 3, 9, 0),
    "l9_3x3_768_512": (512, 256, 512, 3, 9, 0),
}


def run(name, B, reps, inner=20, bf16=False):
    cin1, cin2, cout, k, H, mode = SHAPES[name]
    g = torch.Generator(device="cuda").manual_seed(0)
    hs = H // 2 if mode == 1 else H
    x = torch.randn(B, cin1, hs, hs, device="cuda", generator=g)
    x2 = torch.randn(B, cin2, H, H, device="cuda", generator=g) if cin2 else None
    w = torch.randn(cout, cin1 + cin2, k, k, device="cuda", generator=g) * 0.05
    b = torch.randn(cout, device="cuda", generator=g)
    f = lambda: torch.ops.red_diffeq.conv2d_mfma(x, x2, w, b, None, k // 2, mode, bf16)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(inner):
            f()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * inner)
    flop = 2.0 * B * H * H * cout * (cin1 + cin2) * k * k
    peak = 2500.0 if bf16 else 157.3
    return {"shape": name, "B": B, "bf16": bf16, "us": round(us, 2), "tflops": round(flop / us / 1e6, 1),
            "mfma_frac": round(flop / us / 1e6 / peak, 3)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, nargs="+", default=[1])
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--inner", type=int, default=20)
    ap.add_argument("--f32-min-tiles", type=int, nargs="+", default=[None])
    ap.add_argument("--opt", type=int, default=None, help="another rdq_unet_set_option option id to compare")
    ap.add_argument("--opt-values", type=int, nargs="+", default=[None], help="... and its values")
    a = ap.parse_args()
    names = [a.only] if a.only else list(SHAPES)
    for B in a.B:
        for n in names:
            for ft in a.f32_min_tiles:
              for ov in a.opt_values:
                old = None if ft is None else _hip.lib().rdq_unet_set_option(4, ft)
                old_o = None if ov is None else _hip.lib().rdq_unet_set_option(a.opt, ov)
                try:
                    r = run(n, B, a.reps, a.inner, a.bf16)
                    if ov is not None:
                        r["opt"], r["opt_value"] = a.opt, ov
                finally:
                    if old is not None:
                        _hip.lib().rdq_unet_set_option(4, old)
                    if old_o is not None:
                        _hip.lib().rdq_unet_set_option(a.opt, old_o)
                if ft is not None:
                    r["f32_min_tiles"] = ft
                print(json.dumps(r), flush=True)
