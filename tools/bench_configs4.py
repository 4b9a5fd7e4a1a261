"""configs[4] RED-DiffEq iteration on one MI355X (new behaviour: the reference has no path for a
500 x 3000 model): 16 shots of the 128-shot survey (the per-GPU share of the 8-way sharding),
nt = 1000, the 2-D tiled patch regulariser (70 x 70 tiles placed by calculate_patches along both
axes, one batched U-Net call) with the U-Net convolutions in fp32 or bf16 (mixed precision: bf16
operands, fp32 accumulation), Adam + clamp + metrics through the drop-in InversionEngine.

Prints one JSON line per precision: ms per iteration (mean over iterations [warmup, warmup+iters)),
the U-Net batch (tiles), the U-Net forward alone on that batch, and the bf16 U-Net's relative L2
deviation from fp32 on the same tiles.
python tools/bench_configs4.py [--ns 16] [--iters 3] [--warmup 1] [--nz 500] [--nx 3000]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.core.inversion import InversionEngine  # noqa: E402
from red_diffeq.models.diffusion import GaussianDiffusion, Unet  # noqa: E402
from red_diffeq.regularization.diffusion import tile_plan  # noqa: E402
from red_diffeq.solvers.pde import FWIForward  # noqa: E402
from red_diffeq.utils.data_trans import (prepare_initial_model, s_normalize_none, v_denormalize,  # noqa: E402
                                         v_normalize)
from red_diffeq.utils.ssim import SSIM  # noqa: E402
from red_diffeq.utils.synthetic import make_model  # noqa: E402

UNET_GFLOP = 18.167      # conv FLOP per 72x72 sample, reference architecture

ap = argparse.ArgumentParser()
ap.add_argument("--ns", type=int, default=16)
ap.add_argument("--nz", type=int, default=500)
ap.add_argument("--nx", type=int, default=3000)
ap.add_argument("--nt", type=int, default=1000)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--warmup", type=int, default=1)
ap.add_argument("--precision", type=str, default="fp32,bf16")
ap.add_argument("--unet-only", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(8888)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250, objective="pred_noise").to(dev)
diff.eval()
tp = tile_plan(a.nz, a.nx, 70, 1, dev)
precs = a.precision.split(",")

# the U-Net alone on one iteration's tile batch, and the bf16 deviation from fp32 on it
x = torch.randn(tp.P, 1, 72, 72, device=dev).clamp(-1, 1)
t = torch.randint(0, 1000, (tp.P,), device=dev)
unet = {}
with torch.no_grad():
    for p in precs:
        net.set_precision(p)
        out = net(x, t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            out = net(x, t)
        torch.cuda.synchronize()
        unet[p] = ((time.perf_counter() - t0) / 3 * 1e3, out)
dev_rel = None
if "fp32" in unet and "bf16" in unet:
    ref, got = unet["fp32"][1], unet["bf16"][1]
    dev_rel = float((got - ref).norm() / ref.norm())
for p in precs:
    print(json.dumps({"unet_precision": p, "unet_tiles": tp.P, "unet_forward_ms": round(unet[p][0], 2),
                      "unet_conv_tflops": round(UNET_GFLOP * tp.P / unet[p][0], 1),
                      "bf16_vs_fp32_rel_l2": dev_rel}), flush=True)
if a.unet_only:
    sys.exit(0)

ctx = dict(n_grid=a.nx, nt=a.nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=a.nx, ns=a.ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
vt = torch.from_numpy(make_model("curvefault", a.nz, a.nx, seed=8888, batch=1))
with torch.no_grad():
    y = fwi(v_normalize(vt).to(dev))
mu = torch.nn.functional.pad(prepare_initial_model(vt, "smoothed", sigma=10.0), (1, 1, 1, 1))
for p in precs:
    net.set_precision(p)
    eng = InversionEngine(diff, SSIM(), regularization="diffusion", sigma_x0=1e-4, show_progress=False)

    def run(ts):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.optimize(mu, vt, y, fwi, ts=ts, lr=0.03, reg_lambda=0.75, regularization="diffusion")
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(1)                      # one-off setup (plans, buffers, graph captures) outside both timings
    t_w = run(a.warmup)
    t_all = run(a.warmup + a.iters)
    ms = (t_all - t_w) / a.iters * 1e3
    print(json.dumps({"workload": f"configs[4]: {a.nz}x{a.nx} model, {a.ns} shots/GPU, nt={a.nt}, RED-DiffEq "
                                  "iteration (fwd+adj + 2-D tiled U-Net regulariser + Adam + metrics)",
                      "unet_precision": p, "ms_per_iter": round(ms, 1),
                      "shot_ts_per_s": round(a.ns * a.nt / (ms * 1e-3)), "unet_tiles": tp.P}), flush=True)
