"""A/B of the halo-staged 3x3 convs' options: least tile count of the bf16 kernel
(RDQ_UNET_OPT_CONV3_MIN_TILES), raw conv output held as bf16 (RDQ_UNET_OPT_BF16_RAW) and least tile count
of the fp32 kernel (RDQ_UNET_OPT_CONV3F_MIN_TILES, 0 = off); times the U-Net forward (dim 64, mults
1,2,4,8, 72x72) for each combination and reports the output difference against the first one.
python tools/conv3_threshold_ab.py [--B 344] [--precision bf16] [--min-tiles 512 128] [--f32-min-tiles 0 128]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq import _hip  # noqa: E402
from red_diffeq.models.diffusion import Unet  # noqa: E402

OPT_CONV3_MIN_TILES = 2
OPT_BF16_RAW = 3
OPT_CONV3F_MIN_TILES = 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, nargs="+", default=[344])
    ap.add_argument("--min-tiles", type=int, nargs="+", default=[64])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bf16-raw", type=int, nargs="+", default=[1],
                    help="RDQ_UNET_OPT_BF16_RAW values to A/B (raw conv output held as bf16 or fp32)")
    ap.add_argument("--f32-min-tiles", type=int, nargs="+", default=[-1], help="-1: the library default")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--fused-la-f32", default=None, choices=["auto", "on", "off"],
                    help="unet_ops.FUSED_LA_F32 for this run (default: the module's)")
    a = ap.parse_args()
    if a.fused_la_f32:
        from red_diffeq.models import unet_ops
        unet_ops.FUSED_LA_F32 = {"auto": None, "on": True, "off": False}[a.fused_la_f32]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(dev).eval()
    net.set_precision(a.precision)
    lib = _hip.lib()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for B in a.B:
        x = torch.randn(B, 1, 72, 72, device=dev).clamp(-1, 1)
        t = torch.randint(0, 1000, (B,), device=dev)
        base = None
        for mt, raw, ft in [(m, r, f) for m in a.min_tiles for r in a.bf16_raw for f in a.f32_min_tiles]:
            net.__dict__.pop("_graphs", None)          # small batches replay a captured graph: recapture
            old_raw = lib.rdq_unet_set_option(OPT_BF16_RAW, raw)
            old_ft = lib.rdq_unet_set_option(OPT_CONV3F_MIN_TILES, 0)
            lib.rdq_unet_set_option(OPT_CONV3F_MIN_TILES, old_ft if ft < 0 else ft)
            old = lib.rdq_unet_set_option(OPT_CONV3_MIN_TILES, mt)
            assert old > 0
            try:
                with torch.no_grad():
                    for _ in range(2):
                        y = net(x, t)
                    torch.cuda.synchronize()
                    ts = []
                    for _ in range(a.reps):
                        ev[0].record()
                        y = net(x, t)
                        ev[1].record()
                        torch.cuda.synchronize()
                        ts.append(ev[0].elapsed_time(ev[1]))
            finally:
                lib.rdq_unet_set_option(OPT_CONV3_MIN_TILES, old)
                lib.rdq_unet_set_option(OPT_BF16_RAW, old_raw)
                lib.rdq_unet_set_option(OPT_CONV3F_MIN_TILES, old_ft)
            if base is None:
                base = y.clone()
            d = ((y - base).abs().max() / base.abs().max()).item()
            print(json.dumps({"B": B, "precision": a.precision, "min_tiles": mt, "bf16_raw": raw, "f32_min_tiles": ft, "ms_median": round(sorted(ts)[len(ts) // 2], 3),
                              "ms_min": round(min(ts), 3), "rel_diff_vs_first": d}), flush=True)


if __name__ == "__main__":
    main()
