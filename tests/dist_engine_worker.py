"""One rank of the sharded InversionEngine on the HIP path (tests/test_gpu_sharding.py launches it
with torch.distributed.run).  Every rank uses cuda:0 of the one-GPU test box and the gloo backend
(RCCL needs one GPU per rank; gloo all-reduces device tensors through the host), so this checks the
product's sharded engine end to end on the real kernels; the driver's 8-GPU runs use RCCL.

Usage: python -m torch.distributed.run --nproc-per-node N tests/dist_engine_worker.py OUT.npz
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "red-diffeq_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from conftest import ctx_of, load_golden, replay_draws  # noqa: E402


def main(out):
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
    from red_diffeq.utils.ssim import SSIM
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    backend = os.environ.get("RDQ_TEST_BACKEND", "gloo")
    if backend == "nccl":      # RCCL, initialised the way bench.py does (one rank per GPU: world size 1 here)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    z = load_golden("loop_noise_small")
    ctx = ctx_of(z)
    ns = int(ctx["ns"])
    shots = (rank * ns // world, (rank + 1) * ns // world)
    fwi = FWIForward(dict(ctx), dev, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none,
                     shots=shots)

    class dm:
        device = dev
    ts, lr, lam, sigma, missing, noise_std = z["params"]
    eng = InversionEngine(dm, SSIM(window_size=11), "tv", show_progress=False)
    # record that the engine took its sharded branch: grad_all_reduce's backward ran (with the fault word)
    from red_diffeq.core import inversion as inv
    eng_sharded = [False]
    orig = inv._GradAllReduce.backward

    def backward(ctx, g):
        eng_sharded[0] = ctx.monitor is not None
        return orig(ctx, g)
    inv._GradAllReduce.backward = staticmethod(backward)
    with replay_draws(z):
        mu, hist = eng.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]),
                                torch.from_numpy(z["y"]).to(dev), fwi, ts=int(ts), lr=float(lr), reg_lambda=float(lam),
                                missing_number=int(missing), noise_std=float(noise_std),
                                noise_type=str(z["noise_type"]), regularization="tv")
    mu = mu.detach().cpu().numpy()
    gathered = [torch.zeros(mu.size, dtype=torch.float64) for _ in range(world)]
    if backend == "nccl":
        gathered = [torch.from_numpy(mu.astype(np.float64).ravel())]   # (one rank; RCCL gathers device tensors)
    else:
        dist.all_gather(gathered, torch.from_numpy(mu.astype(np.float64).ravel()))
    if rank == 0:
        np.savez(out, mu=mu, same=np.array(all(torch.equal(g, gathered[0]) for g in gathered)),
                 backend=np.array(dist.get_backend()), sharded=np.array(bool(eng_sharded[0])),
                 **{k: np.array([h[k] for h in hist]) for k in hist[0]})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
