"""Where the reference notebook configuration's iteration goes (CurveFault, ns = 5, nt = 1000): the
InversionEngine loop with the diffusion regulariser (U-Net on the side stream, and with
RDQ_NO_OVERLAP=1 serialised) against the same loop with regularization "tv" and "none" (the FWI
floor).  python tools/notebook_floor.py [steps] [regs, e.g. diffusion,none] -> one JSON line (ms per
iteration)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "red-diffeq_amd")]
import torch  # noqa: E402


def make_loop(dev, reg, ns=5):
    """run(ts, sync=True) -> seconds of one InversionEngine.optimize call of ts iterations."""
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.ssim import SSIM
    from red_diffeq.utils.synthetic import make_model
    torch.manual_seed(8888)
    ctx = dict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=ns)
    fwi = FWIForward(dict(ctx), dev, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    vt = torch.from_numpy(make_model("curvefault", 70, 70, seed=8888, batch=1))
    with torch.no_grad():
        y = fwi(v_normalize(vt).to(dev))
    mu = torch.nn.functional.pad(prepare_initial_model(vt, "smoothed", sigma=10.0), (1, 1, 1, 1))
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
    diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                             objective="pred_noise").to(dev)
    reg = None if reg == "none" else reg
    eng = InversionEngine(diff, SSIM(), regularization=reg, sigma_x0=1e-4, show_progress=False)

    # RDQ_MAIN_PRIO=1: the whole loop on a high-priority stream (the FWI and its serial tail ahead of
    # the side stream's U-Net kernels at every dispatch)
    hp = torch.cuda.Stream(device=dev, priority=-1) if os.environ.get("RDQ_MAIN_PRIO") else None

    def run(ts, sync=True):
        if sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        if hp is not None:
            hp.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(hp):
                eng.optimize(mu, vt, y, fwi, ts=ts, lr=0.03, reg_lambda=0.75, regularization=reg)
            torch.cuda.current_stream(dev).wait_stream(hp)
        else:
            eng.optimize(mu, vt, y, fwi, ts=ts, lr=0.03, reg_lambda=0.75, regularization=reg)
        if sync:
            torch.cuda.synchronize()
        return time.perf_counter() - t0

    return run


def loop_ms(dev, reg, ns=5, steps=20, warmup=3):
    run = make_loop(dev, reg, ns)
    run(1)
    t_w = run(warmup)
    t_all = run(warmup + steps)
    return round((t_all - t_w) / steps * 1e3, 3)


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    regs = sys.argv[2].split(",") if len(sys.argv) > 2 else ("diffusion", "tv", "none")
    out = {k: loop_ms(dev, k, steps=steps) for k in regs}
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("RDQ_")}
    print(json.dumps(out), flush=True)
