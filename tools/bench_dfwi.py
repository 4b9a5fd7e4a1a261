"""DiffusionFWI baseline (diffusion_bench) timing on one MI355X at the reference's OpenFWI setting:
70x70 model, ns=5, nt=1000, dim-64 U-Net (random init: no checkpoint offline).  Reports ms per
reverse-diffusion step with `ts` inner FWI iterations (denoise + ts x (fwd + L1 + adj + Adam) +
metrics) and the inner-iteration rate.
python tools/bench_dfwi.py [--ts 10] [--diffusion-ts 6] [--ns 5]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from diffusion_bench import DiffusionFWI  # noqa: E402
from red_diffeq.models.diffusion import GaussianDiffusion, Unet  # noqa: E402
from red_diffeq.solvers.pde import FWIForward  # noqa: E402
from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize  # noqa: E402
from red_diffeq.utils.ssim import SSIM  # noqa: E402
from red_diffeq.utils.synthetic import make_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ts", type=int, default=10)
ap.add_argument("--diffusion-ts", type=int, default=6)
ap.add_argument("--ns", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(8888)
ctx = dict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=a.ns)
fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
vt = torch.from_numpy(make_model("curvefault", 70, 70, seed=8888, batch=1))
with torch.no_grad():
    y = fwi(v_normalize(vt).to(dev))
mu0 = prepare_initial_model(vt, "smoothed", sigma=10.0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250, objective="pred_noise").to(dev)
bench = DiffusionFWI(diff.eval(), fwi, SSIM())


def run(dts):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bench.optimize(mu0, vt, y, fwi, ts=a.ts, diffusion_ts=dts, lr=0.03)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


run(2)
t1 = run(1)                       # the t = 0 step only: denoise + metrics, no FWI
tn = run(a.diffusion_ts)
per_step = (tn - t1) / (a.diffusion_ts - 1) * 1e3
print(json.dumps({"workload": f"DiffusionFWI (diffusion_bench), OpenFWI CurveFault 70x70, ns={a.ns}, nt=1000, "
                              f"ts={a.ts} inner FWI iterations per reverse step, random-init dim-64 U-Net",
                  "ms_per_reverse_step": round(per_step, 2),
                  "ms_per_inner_fwi_iteration": round(per_step / a.ts, 3),
                  "shot_ts_per_s": round(a.ns * 1000 * a.ts / (per_step * 1e-3))}), flush=True)
