"""fp32 LinearAttention block: the fused two-launch form (rdq_linear_attention_f32) against the unfused
path (to_qkv with RMSNorm, context, output block) per U-Net level and batch, device time per call from a
replayed hipGraph of back-to-back calls (the U-Net's own launch conditions).
python tools/la_f32_ab.py [--B 1 8 25 100 344]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.models import unet_ops  # noqa: E402
from red_diffeq.models.diffusion import LinearAttention  # noqa: E402

LEVELS = [(64, 72), (64, 36), (128, 36), (128, 18)]      # (dim, H): the fusable blocks of the dim-64 U-Net


def time_us(fn, inner=5, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (inner * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, nargs="+", default=[1, 8, 25, 100, 344])
    a = ap.parse_args()
    torch.manual_seed(0)
    for B in a.B:
        for dim, H in LEVELS:
            m = LinearAttention(dim).cuda().eval()
            x = torch.randn(B, dim, H, H, device="cuda")
            res = {}
            with torch.no_grad():
                for fused in (False, True):
                    unet_ops.FUSED_LA_F32 = fused
                    res[fused] = (time_us(lambda: unet_ops.linear_attention(x, m)), unet_ops.linear_attention(x, m))
            unet_ops.FUSED_LA_F32 = False
            d = ((res[True][1] - res[False][1]).abs().max() / res[False][1].abs().max()).item()
            print(json.dumps({"B": B, "dim": dim, "H": H, "unfused_us": round(res[False][0], 1),
                              "fused_us": round(res[True][0], 1), "rel_diff": d}), flush=True)


if __name__ == "__main__":
    main()
