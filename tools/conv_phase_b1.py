"""Where a B = 1 U-Net conv launch spends its time: per-workgroup s_memrealtime stamps (10 ns) recorded by a
timing-only build of the library (tools/exp_build.py --src unet cprof ..., selected with RDQ_HIP_LIB; the
product library has no stamps) at conv_cc_seg's phase points: entry -> first stage staged (t1) -> K loop
done (t2) -> split-K combine done (t3) -> outputs stored (t4) -> GroupNorm partials stored (t5).
Records of the last-arriving split only (the tile's critical path).  Per launch also the span from the
first workgroup's entry to the last one's exit, and the gap to the next launch's first entry.
python tools/conv_phase_b1.py [reps]"""
import ctypes
import json
import os
import sys
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq import _hip  # noqa: E402
from red_diffeq.models.diffusion import Unet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
lib = _hip.lib()
fn = lib.rdq_exp_cprof
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
x = torch.randn(1, 1, 72, 72, device="cuda")
t = torch.randint(0, 1000, (1,), device="cuda")
buf = np.zeros((65536, 8), np.uint64)
with torch.no_grad():
    xs, ts = net.graph_io(x.shape, x.device)
    xs.copy_(x)
    ts.copy_(t)
    for _ in range(3):
        net.replay_static(xs, ts)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, 65536, 1)
    per = defaultdict(list)
    spans = defaultdict(list)
    for _ in range(reps):
        net.replay_static(xs, ts)
        torch.cuda.synchronize()
        n = fn(buf.ctypes.data, 65536, 1)
        r = buf[:n].astype(np.int64)
        r = r[np.argsort(r[:, 1], kind="stable")]
        # launches: consecutive records (by entry time); a new launch once an entry follows every exit so far
        groups, cur, cur_end = [], [], -1
        for row in r:
            if cur and row[1] > cur_end:
                groups.append(np.array(cur))
                cur, cur_end = [], -1
            cur.append(row)
            cur_end = max(cur_end, row[6])
        if cur:
            groups.append(np.array(cur))
        for gi, g in enumerate(groups):
            key = int(g[0, 0])
            H, cout, cin, taps, gn = key >> 48, (key >> 32) & 0xffff, (key >> 16) & 0xffff, (key >> 8) & 0xff, key & 1
            name = f"{H}x{H} {cin}->{cout} k{taps}{' gn' if gn else ''} S{int(g[0, 7])}"
            ph = np.diff(g[:, 1:7], axis=1) / 100.0            # us per phase, per workgroup
            per[name].append(np.median(ph, axis=0))
            nxt = groups[gi + 1][:, 1].min() if gi + 1 < len(groups) else None
            spans[name].append(((g[:, 6].max() - g[:, 1].min()) / 100.0,
                                (nxt - g[:, 6].max()) / 100.0 if nxt is not None else np.nan, len(g)))
out = []
for name in per:
    ph = np.median(np.array(per[name]), axis=0)
    sp = np.array(spans[name])
    out.append({"conv": name, "launches_per_forward": len(per[name]) // reps,
                "median_phase_us": {"stage0": round(ph[0], 2), "kloop": round(ph[1], 2), "combine": round(ph[2], 2),
                                    "epilogue_store": round(ph[3], 2), "gn_partials": round(ph[4], 2)},
                "wg_span_us": round(float(np.median(sp[:, 0])), 2), "gap_to_next_conv_us": round(float(np.nanmedian(sp[:, 1])), 2),
                "records": int(np.median(sp[:, 2]))})
for o in sorted(out, key=lambda o: -o["wg_span_us"] * o["launches_per_forward"]):
    print(json.dumps(o))
