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


def test_shot_slice_helper():
    from red_diffeq.core.inversion import shot_slice

    class F:
        shots = (0, 8)
    assert shot_slice(F(), 8) is None
    F.shots = (2, 5)
    assert shot_slice(F(), 8) == (2, 5)
