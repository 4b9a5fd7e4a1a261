"""Where a k_conv3_bf16 workgroup spends its life (timing-only build from tools/exp_c3prof.py, selected with
RDQ_HIP_LIB=red-diffeq_amd/lib_exp/libc3prof.so): per-workgroup stamps at entry, chunk 0 staged (first barrier),
taps done, epilogue done.  One launch of each conv_micro shape named (default l72_3x3_64_64 at B = 344),
median phase durations (us), the launch span and the mean number of workgroups resident per CU.
python tools/c3_phase.py [SHAPE ...] [--B 344]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from red_diffeq import _hip  # noqa: E402
import conv_micro  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("shapes", nargs="*", default=["l72_3x3_64_64"])
ap.add_argument("--B", type=int, default=344)
ap.add_argument("--unet", action="store_true", help="the stamps of the bf16 U-Net forward's LAST halo conv (72 x 72, 64 out)")
a = ap.parse_args()
lib = _hip.lib()
fn = lib.rdq_exp_c3prof
fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
ncu = torch.cuda.get_device_properties(0).multi_processor_count
if a.unet:
    from red_diffeq.models.diffusion import Unet  # noqa: E402
    torch.manual_seed(0)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
    net.set_precision("bf16")
    x = torch.randn(a.B, 1, 72, 72, device="cuda").clamp(-1, 1)
    tt = torch.randint(0, 1000, (a.B,), device="cuda")
    res = []
    nwg = (a.B * 72 * 72 + 255) // 256
    with torch.no_grad():
        for rep in range(6):
            net(x, tt)
            torch.cuda.synchronize()
            buf = np.zeros((nwg, 4), np.uint64)
            assert fn(buf.ctypes.data, nwg) == 0
            t = buf.astype(np.int64)
            t -= t[:, 0].min()
            ph = np.diff(t, axis=1) / 100.0
            life = (t[:, 3] - t[:, 0]) / 100.0
            span = t[:, 3].max() / 100.0
            if rep >= 2:
                res.append({"prologue": np.median(ph[:, 0]), "taps": np.median(ph[:, 1]), "epilogue": np.median(ph[:, 2]),
                            "life": np.median(life), "span": span, "resident_per_cu": life.sum() / span / ncu, "nwg": nwg})
    out = {"shape": "unet_bf16_last_halo_conv_l72", "B": a.B}
    for key in res[0]:
        out[key] = round(float(np.median([r[key] for r in res])), 3)
    print(json.dumps(out), flush=True)
for name in ([] if a.unet else a.shapes):
    cin1, cin2, cout, k, H, mode = conv_micro.SHAPES[name]
    g = torch.Generator(device="cuda").manual_seed(0)
    hs = H // 2 if mode == 1 else H
    x = torch.randn(a.B, cin1, hs, hs, device="cuda", generator=g)
    x2 = torch.randn(a.B, cin2, H, H, device="cuda", generator=g) if cin2 else None
    w = torch.randn(cout, cin1 + cin2, k, k, device="cuda", generator=g) * 0.05
    b = torch.randn(cout, device="cuda", generator=g)
    res = []
    for rep in range(6):
        torch.ops.red_diffeq.conv2d_mfma(x, x2, w, b, None, k // 2, mode, True)
        torch.cuda.synchronize()
        nwg = (a.B * H * H + 255) // 256 * (cout // 64)
        buf = np.zeros((min(nwg, 65536), 4), np.uint64)
        assert fn(buf.ctypes.data, buf.shape[0]) == 0
        t = buf.astype(np.int64)
        t -= t[:, 0].min()
        ph = np.diff(t, axis=1) / 100.0
        life = (t[:, 3] - t[:, 0]) / 100.0
        span = (t[:, 3].max()) / 100.0
        if rep >= 2:
            res.append({"prologue": np.median(ph[:, 0]), "taps": np.median(ph[:, 1]), "epilogue": np.median(ph[:, 2]),
                        "life": np.median(life), "span": span, "resident_per_cu": life.sum() / span / ncu,
                        "nwg": int(nwg)})
    out = {"shape": name, "B": a.B}
    for key in res[0]:
        out[key] = round(float(np.median([r[key] for r in res])), 3)
    print(json.dumps(out), flush=True)
