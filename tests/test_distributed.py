"""Shot-parallel data parallelism on CPU with the gloo backend, world sizes 2 and 3.

Each rank models a contiguous block of shots; the data-term gradient is summed by ONE
all-reduce inside backward (red_diffeq.core.inversion.grad_all_reduce) and the misfit is
normalised by the global observation count.  The FWI operator here is the oracle wrapped as an
autograd Function (test infrastructure; the product operator is the HIP one), which exercises the
product's sharding and reduction logic exactly as InversionEngine applies it.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, ctx_of, load_golden, vnorm

CTX = None


class _OracleOp(torch.autograd.Function):
    @staticmethod
    def forward(c, v, f):
        seis, cf = f.forward(v.detach().contiguous().numpy().astype(np.float32), keep_history=True)
        c.f, c.cf = f, cf
        return torch.from_numpy(seis)

    @staticmethod
    def backward(c, g):
        gA, gK, gb = c.f.adjoint(c.cf, g.contiguous().numpy())
        return torch.from_numpy(c.f.finalize(c.cf, gA, gK, gb)), None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_grad(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
    from oracle import oracle as O
    from red_diffeq.core.inversion import grad_all_reduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    z = load_golden("grad_small")
    ctx = ctx_of(z)
    ns = 3
    shots = {2: [(0, 2), (2, 3)], 3: [(0, 1), (1, 2), (2, 3)]}[world][rank]   # uneven at world 2
    import numpy as _np
    from oracle.oracle import geometry
    isx, isz, igx, igz = geometry(ctx)
    sub = dict(ctx)
    sub["sx"] = list(((isx[shots[0]:shots[1]] - ctx["nbc"]).astype(float)))
    f = O.OracleFWI(sub, 2)
    v = torch.from_numpy(vnorm(z["v_init"])).requires_grad_(True)
    y = torch.from_numpy(z["y"][:, shots[0]:shots[1]])
    # global observation count (all ones here): one all-reduce, as the engine does
    nobs_local = torch.full((2,), float(y[0].numel()))
    nobs = nobs_local.clone()
    dist.all_reduce(nobs)
    vin = grad_all_reduce(v)
    pred = _OracleOp.apply(vin, f)
    loss = ((y - pred).abs().reshape(2, -1).sum(1, dtype=torch.float64) / nobs.double()).float()
    tv = (v[:, :, :, 1:] - v[:, :, :, :-1]).abs().flatten(1).mean(1)   # replicated term
    (loss + 0.01 * tv).sum().backward()
    obs = loss.detach().clone()
    dist.all_reduce(obs)
    if rank == 0:
        out["grad"] = v.grad.numpy().copy()
        out["loss"] = obs.numpy().copy()
    dist.barrier()
    dist.destroy_process_group()
    del _np, ns


def _worker(rank, world, port, q):
    out = {}
    _sharded_grad(rank, world, port, out)
    if rank == 0:
        q.put(out)


@pytest.mark.parametrize("world", [2, 3])
def test_shot_parallel_gradient_equals_single_rank(world):
    from oracle import oracle as O
    z = load_golden("grad_small")
    ctx = ctx_of(z)
    f = O.OracleFWI(ctx, 2)
    v = torch.from_numpy(vnorm(z["v_init"])).requires_grad_(True)
    y = torch.from_numpy(z["y"])
    pred = _OracleOp.apply(v, f)
    loss = ((y - pred).abs().reshape(2, -1).sum(1, dtype=torch.float64) / float(y[0].numel())).float()
    tv = (v[:, :, :, 1:] - v[:, :, :, :-1]).abs().flatten(1).mean(1)
    (loss + 0.01 * tv).sum().backward()
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    ps = [ctxm.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_allclose(out["loss"], loss.detach().numpy(), rtol=1e-6)
    g1 = v.grad.numpy()
    rel = np.linalg.norm(out["grad"] - g1) / np.linalg.norm(g1)
    assert rel < 1e-5, rel


# ------------------------------------------------------------------ the sharded InversionEngine
def _install_cpu_standins(setattr_=setattr):
    """Run InversionEngine.optimize on CPU: its device kernels (fused Adam + clamp K11, fused
    metrics K12, L1 misfit K5, TV K6) are replaced by plain torch restatements of the same
    contracts, so the engine's OWN sharding logic (shot_slice, the global observation count, y /
    mask slicing, grad_all_reduce, the obs-loss all-reduce) runs unchanged under gloo.  Test
    infrastructure only: the product refuses CPU tensors."""
    import red_diffeq.core.inversion as inv
    import red_diffeq.core.losses as losses
    import red_diffeq.regularization.base as base
    from red_diffeq.utils.ssim import SSIM

    class TorchAdamClamp:
        def __init__(self, param, lr, betas=(0.9, 0.999), eps=1e-8, clamp=(-1.0, 1.0)):
            self.param, self.clamp, self.t = param, clamp, 0
            self.opt = torch.optim.Adam([param], lr=lr, betas=betas, eps=eps)

        @property
        def lr(self):
            return self.opt.param_groups[0]["lr"]

        @lr.setter
        def lr(self, v):
            self.opt.param_groups[0]["lr"] = v

        def zero_grad(self):
            self.opt.zero_grad(set_to_none=True)

        def step(self, guard=None):
            self.t += 1
            self.opt.step()
            with torch.no_grad():
                self.param.clamp_(*self.clamp)

    ssim = SSIM(window_size=11)

    def torch_metrics(pred, true_norm):
        d = pred.detach() - true_norm
        mae = d.abs().mean(dim=(1, 2, 3))
        rmse = (d ** 2).mean(dim=(1, 2, 3)).sqrt()
        ss = torch.stack([ssim((pred[i:i + 1].detach() + 1) / 2, (true_norm[i:i + 1] + 1) / 2)
                          for i in range(pred.shape[0])])
        return torch.stack([mae, rmse, ss])

    class TorchL1(torch.autograd.Function):
        @staticmethod
        def forward(ctx, pred, y, mask, nobs_override):
            m = torch.ones_like(pred) if mask is None else mask
            nobs = m.flatten(1).sum(1).clamp(min=1.0) if nobs_override is None else nobs_override
            ctx.save_for_backward(pred, y, m, nobs)
            return ((y - pred).abs() * m).flatten(1).sum(1) / nobs

        @staticmethod
        def backward(ctx, g):
            pred, y, m, nobs = ctx.saved_tensors
            return torch.sign(pred - y) * m * (g / nobs).view(-1, 1, 1, 1), None, None, None

    def torch_tv(mu):
        return (mu[:, :, :, 1:] - mu[:, :, :, :-1]).abs().flatten(1).mean(1) + \
            (mu[:, :, 1:, :] - mu[:, :, :-1, :]).abs().flatten(1).mean(1)

    setattr_(inv, "FusedAdamClamp", TorchAdamClamp)
    setattr_(inv, "fused_metrics", torch_metrics)
    setattr_(losses, "_L1Misfit", TorchL1)
    setattr_(base, "total_variation_loss", torch_tv)


class _OracleShotOp:
    """The oracle (CPU restatement of FWIForward) modelling shots [a, b) of the survey, with the
    drop-in operator's surface: callable, .to(device), .shots."""

    def __init__(self, ctx, B, shots):
        from oracle import oracle as O
        from oracle.oracle import geometry
        isx = geometry(ctx)[0]
        sub = dict(ctx)
        sub["sx"] = list((isx[shots[0]:shots[1]] - ctx["nbc"]).astype(float))
        self.f = O.OracleFWI(sub, B)
        self.shots = shots

    def to(self, device):
        return self

    def __call__(self, v):
        return _OracleOp.apply(v, self.f)


def _engine_run(ctx, z, shots, group=None):
    from conftest import replay_draws
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.utils.ssim import SSIM

    class dm:
        device = torch.device("cpu")
    ts, lr, lam, sigma, missing, noise_std = z["params"]
    eng = InversionEngine(dm, SSIM(window_size=11), "tv", show_progress=False)
    with replay_draws(z):      # the reference's noise / missing-receiver draws, identical on every rank
        mu, hist = eng.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]), torch.from_numpy(z["y"]),
                                _OracleShotOp(ctx, z["mu0"].shape[0], shots), ts=int(ts), lr=float(lr),
                                reg_lambda=float(lam), missing_number=int(missing), noise_std=float(noise_std),
                                noise_type=str(z["noise_type"]), regularization="tv", process_group=group)
    return mu.detach().numpy(), {k: np.array([h[k] for h in hist]) for k in hist[0]}


def _engine_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    _install_cpu_standins()
    z = load_golden("loop_noise_small")
    ns = int(z["ctx_ns"])
    shots = (rank * ns // world, (rank + 1) * ns // world)     # world 2: (0, 1), (1, 3)
    mu, hist = _engine_run(ctx_of(z), z, shots)
    if rank == 0:
        q.put((mu, hist))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_inversion_engine_equals_single_rank(monkeypatch):
    """InversionEngine.optimize end to end with shot-sharded operators over gloo (world 2, uneven
    split 1 + 2 of 3 shots, B = 2 models, Gaussian noise + 4 missing receivers replayed from the
    reference's draws): the engine's sharded branch (shot_slice, global_nobs from the replicated
    mask, y / mask slices, grad_all_reduce, the obs-loss all-reduce) gives the single-rank result."""
    _install_cpu_standins(monkeypatch.setattr)      # undone after the test
    z = load_golden("loop_noise_small")
    ns = int(z["ctx_ns"])
    mu1, h1 = _engine_run(ctx_of(z), z, (0, ns))
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    ps = [ctxm.Process(target=_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    mu2, h2 = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = np.sqrt(np.mean((mu2.astype(np.float64) - mu1) ** 2))
    assert d < 1e-5, d
    for k in ("obs_losses", "total_losses", "rmse"):
        np.testing.assert_allclose(h2[k], h1[k], rtol=1e-5, err_msg=k)
    # and the single-rank CPU engine itself follows the reference's trajectory
    np.testing.assert_allclose(h1["obs_losses"], z["obs_losses"], rtol=1e-4)


def test_shot_slice_helper():
    from red_diffeq.core.inversion import shot_slice

    class F:
        shots = (0, 8)
    assert shot_slice(F(), 8) is None
    F.shots = (2, 5)
    assert shot_slice(F(), 8) == (2, 5)
    F.shots, F.shots_explicit = (0, 8), True    # sharding asked for explicitly: kept at one rank too
    assert shot_slice(F(), 8) == (0, 8)
