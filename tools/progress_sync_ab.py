#!/usr/bin/env python
"""InversionEngine.optimize per-iteration wallclock with the rank-0 progress bar on vs off (the
script path, scripts/run_inversion.py, shows it on rank 0).  The bar's postfix reads pinned async
copies behind events (core/inversion.py _Progress), so both should cost the same: no per-iteration
host sync.  TV loop at configs[1] (FlatVel-A, 8 shots, nt 1000) and the RED loop at the reference
notebook's configuration (CurveFault, 5 shots, dim-64 U-Net).  One JSON line per case."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))


def main():
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.ssim import SSIM
    from red_diffeq.utils.synthetic import make_model
    dev = torch.device("cuda", 0)
    for reg, ns, fam in (("tv", 8, "flatvel"), ("diffusion", 5, "curvefault")):
        ctx = dict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=ns)
        fwi = FWIForward(dict(ctx), dev, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
        vt = torch.from_numpy(make_model(fam, 70, 70, seed=8888, batch=1))
        with torch.no_grad():
            y = fwi(v_normalize(vt).to(dev))
        mu = torch.nn.functional.pad(prepare_initial_model(vt, "smoothed", sigma=10.0), (1, 1, 1, 1))
        if reg == "diffusion":
            torch.manual_seed(0)
            dm = GaussianDiffusion(Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1), image_size=72, timesteps=1000,
                                   sampling_timesteps=250, objective="pred_noise").to(dev)
        else:
            class dm:
                device = dev
        res = {"loop": reg, "ns": ns}
        for show in (False, True, False, True):
            eng = InversionEngine(dm, SSIM(), regularization=reg, sigma_x0=1e-4, show_progress=show)

            def run(ts):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.optimize(mu, vt, y, fwi, ts=ts, lr=0.03, reg_lambda=0.75 if reg == "diffusion" else 0.01,
                             regularization=reg)
                torch.cuda.synchronize()
                return time.perf_counter() - t0
            run(3)
            t5, t45 = run(5), run(45)
            res.setdefault("progress_on_ms" if show else "progress_off_ms", []).append(round((t45 - t5) / 40 * 1e3, 4))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
