#!/usr/bin/env python
"""Full-length (ts = 300, the reference default: red_diffeq/core/inversion.py:27,
configs/default.yaml:35) inversion trajectories of the REFERENCE engine, and the ensemble that
measures how far a correct fp32 trajectory can drift from it.  Runs the reference, in this
container only; writes tests/golden/loop_{tv,red}_300.npz and tests/golden/repro_floor_300.json.

Two trajectories (OpenFWI geometry, ns = 2, nt = 1000, lr = 0.03, cosine schedule to 0 at ts):
  tv   FlatVel-A seed 8888, total variation, lambda 0.01;
  red  CurveVel-A seed 8890, RED-DiffEq with the dim-8 U-Net of gen_unet (make_golden._unet_dim8),
       lambda 0.75, sigma_x0 1e-4 (the regulariser draws eps_x0, t, eps every iteration).

Each is run by the reference engine (InversionEngine.optimize, with the reference's own draws) with
several forward operators, every one a correct fp32 implementation of FWIForward (pde.py:61-93):
  ref          the reference operator itself (torch autograd adjoint): the fixture;
  oracle       oracle/fwi_oracle.c (the HIP kernels' summation order, no FMA);
  oracle_fma   the same source built with FMA contraction (oracle/Makefile);
  pershot      the oracle one shot at a time, per-shot gradients summed after the chain rule (what a
               shot-sharded run computes);
  oracle_p1/2  the oracle with its gradient rounded once more (relative 2^-23 jitter, seeded): a
               second rounding per element, the smallest difference two fp32 operators can have.
All members consume the same global-RNG draws (the operator draws nothing), so they differ only in
floating-point rounding.  The per-iteration model RMSE of each member vs the reference is the
envelope a correct fp32 implementation can be held to (tests/test_gpu_loop_parity.py::
test_trajectory_300_within_ensemble).

The RED draws (1 + 1 + 1 per iteration) are not stored: they are regenerated from torch's CPU
generator (seed 1234, the calls' kinds and arguments stored) and checked against per-draw sums.

Run (members are independent processes; the cache is tests/golden/_cache, git-ignored):
  python tests/golden/make_long.py member tv ref      # ... for every member
  python tests/golden/make_long.py combine tv
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CACHE = os.path.join(HERE, "_cache")
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import make_golden as G  # noqa: E402

TS = int(os.environ.get("LONG_TS", "300"))   # override only to smoke-test this script
CTX = dict(G.OPENFWI, ns=2)
RUNS = {
    "tv": dict(family="flatvel", seed=8888, reg="tv", lam=0.01, lr=0.03, sigma=10.0),
    "red": dict(family="curvevel", seed=8890, reg="diffusion", lam=0.75, lr=0.03, sigma=10.0),
}
MEMBERS = ("ref", "oracle", "oracle_fma", "pershot", "oracle_p1", "oracle_p2")
KEEP_EVERY = 10        # reference models stored at iterations 10, 20, ..., 300 (1-based)


class _JitterOp(torch.autograd.Function):
    """Identity forward; backward multiplies the gradient by (1 + 2^-23 xi), xi in {-1, 0, 1}."""

    @staticmethod
    def forward(c, v, rng):
        c.rng = rng
        return v.view_as(v)

    @staticmethod
    def backward(c, g):
        xi = torch.from_numpy(c.rng.integers(-1, 2, size=g.shape).astype(np.float32))
        return g * (1.0 + xi * np.float32(2.0 ** -23)), None


class _Member:
    def __init__(self, name):
        self.name = name
        if name == "ref":
            self.ops = [G.make_fwi(CTX)]
        elif name == "pershot":
            sx = list(np.linspace(0, CTX["n_grid"] - 1, num=CTX["ns"]))
            self.ops = [G._OracleFWI(dict(CTX, ns=1, sx=[s])) for s in sx]
        else:
            op = G._OracleFWI(CTX)
            if name == "oracle_fma":
                from oracle import oracle as O
                op.f = O.OracleFWI(CTX, 1, variant="fma")
            self.ops = [op]
        self.rng = np.random.default_rng(int(name[-1])) if name.startswith("oracle_p") else None

    def to(self, device):
        return self

    def __call__(self, v):
        if self.rng is not None:
            v = _JitterOp.apply(v, self.rng)
        if len(self.ops) == 1:
            return self.ops[0](v)
        return torch.cat([op(v) for op in self.ops], dim=1)     # per-shot gradients summed by autograd


class _ModelTrace:
    """Records mu (interior, after Adam + clamp) at every iteration: the reference engine calls
    scheduler.step() right after the clamp (inversion.py:88-92)."""

    def __init__(self):
        self.models = []

    def __enter__(self):
        cls = torch.optim.lr_scheduler.CosineAnnealingLR
        self.orig = cls.step
        trace = self

        def step(sched, *a, **kw):
            if getattr(sched, "_traced", False):
                p = sched.optimizer.param_groups[0]["params"][0]
                trace.models.append(p.detach()[:, :, 1:-1, 1:-1].numpy().copy())
            sched._traced = True            # the constructor's own step() is not an iteration
            return trace.orig(sched, *a, **kw)
        cls.step = step
        return self

    def __exit__(self, *exc):
        torch.optim.lr_scheduler.CosineAnnealingLR.step = self.orig


class _DrawLog:
    """Records each global-RNG draw's kind, arguments and float64 sum (values are regenerated)."""

    def __init__(self):
        self.rows = []

    def __enter__(self):
        self.orig = {n: getattr(torch, n) for n in ("randn", "randint")}

        def randn(*a, **kw):
            assert kw.get("generator") is None
            r = self.orig["randn"](*a, **kw)
            self.rows.append((0, 0, 0, r.numel(), float(r.double().sum())))
            return r

        def randint(low, high, size, **kw):
            assert kw.get("generator") is None
            r = self.orig["randint"](low, high, size, **kw)
            self.rows.append((1, low, high, r.numel(), float(r.double().sum())))
            return r
        torch.randn, torch.randint = randn, randint
        for n in ("rand", "randperm"):
            setattr(self, "_" + n, getattr(torch, n))
            setattr(torch, n, lambda *a, _n=n, **kw: (_ for _ in ()).throw(AssertionError(f"unexpected {_n}")))
        return self

    def __exit__(self, *exc):
        torch.randn, torch.randint = self.orig["randn"], self.orig["randint"]
        torch.rand, torch.randperm = self._rand, self._randperm


def inputs(kind):
    r = RUNS[kind]
    v_true = G.synthetic.make_model(r["family"], 70, 70, seed=r["seed"], batch=1)
    init = G.ref.data_trans.prepare_initial_model(torch.from_numpy(v_true), "smoothed", sigma=r["sigma"])
    mu0 = torch.nn.functional.pad(init, (1, 1, 1, 1), "constant", 0)
    return v_true, mu0


def run_member(kind, name):
    r = RUNS[kind]
    v_true, mu0 = inputs(kind)
    with torch.no_grad():
        y = G.run_forward(CTX, v_true)          # the reference forward (bit-exact with the oracle's)
    if r["reg"] == "diffusion":
        diff = G.ref.diffusion.GaussianDiffusion(G._unet_dim8(), image_size=72, timesteps=1000,
                                                 sampling_timesteps=250, objective="pred_noise").eval()
    else:
        diff = G._NoDiffusion()
    eng = G.ref.inversion.InversionEngine(diff, G.ref.ssim.SSIM(window_size=11), r["reg"], sigma_x0=1e-4)
    op = _Member(name)
    torch.manual_seed(1234)
    t0 = time.time()
    with _ModelTrace() as tr, _DrawLog() as dl:
        mu, hist = eng.optimize(mu0, torch.from_numpy(v_true), torch.from_numpy(y), op, ts=TS, lr=r["lr"],
                                reg_lambda=r["lam"], regularization=r["reg"])
    models = np.concatenate(tr.models)[:, 0]                      # (TS, 70, 70)
    assert len(models) == TS and np.array_equal(models[-1], mu.detach().numpy()[0, 0])
    keys = ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")
    os.makedirs(CACHE, exist_ok=True)
    np.savez(os.path.join(CACHE, f"{kind}_{name}.npz"), models=models, y=y, v_true=v_true, mu0=mu0.numpy(),
             draws=np.array(dl.rows, np.float64), seconds=np.array(time.time() - t0),
             **{k: np.array(hist[0][k], np.float64).ravel() for k in keys})
    print(f"[{kind}/{name}] {time.time() - t0:.0f}s final model rmse-vs-true {hist[0]['rmse'][-1]}", flush=True)


def regenerate_draws(rows, shape):
    """The reference's draws from torch's CPU generator, re-made from their kinds and arguments."""
    torch.manual_seed(1234)
    out = []
    for kind, low, high, n, s in rows:
        if kind == 0:
            assert n == int(np.prod(shape))
            d = torch.randn(shape)
        else:
            d = torch.randint(int(low), int(high), (int(n),))
        assert float(d.double().sum()) == s
        out.append(d)
    return out


def rmse(a, b):
    return np.sqrt(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2, axis=(-2, -1)))


def combine(kind):
    r = RUNS[kind]
    runs = {m: np.load(os.path.join(CACHE, f"{kind}_{m}.npz")) for m in MEMBERS
            if os.path.exists(os.path.join(CACHE, f"{kind}_{m}.npz"))}
    assert "ref" in runs and len(runs) >= 4, sorted(runs)
    ref = runs["ref"]
    for m, z in runs.items():
        assert np.array_equal(z["draws"], ref["draws"]), m        # same draws in every member
    if len(ref["draws"]):
        regenerate_draws(ref["draws"], (1, 1, 72, 72))
    metrics = ("mae", "rmse", "ssim", "obs_losses")
    rep = {"trajectory": f"{kind}: OpenFWI {r['family']} seed {r['seed']}, ns=2, nt=1000, lr={r['lr']}, "
                         f"lambda={r['lam']}, reg={r['reg']}, ts={TS}",
           "members": sorted(m for m in runs if m != "ref"), "member_seconds": {m: float(z["seconds"])
                                                                               for m, z in runs.items()}}
    per = {m: rmse(z["models"], ref["models"]) for m, z in runs.items() if m != "ref"}
    env = np.max(np.stack(list(per.values())), axis=0)
    rep["model_rmse_vs_ref_per_member_final"] = {m: float(v[-1]) for m, v in per.items()}
    rep["model_rmse_vs_ref_per_member_max"] = {m: float(v.max()) for m, v in per.items()}
    rep["envelope_model_rmse_per_iter"] = env.tolist()
    rep["envelope_final"] = float(env[-1])
    rep["envelope_max"] = float(env.max())
    for k in metrics:
        devs = np.stack([np.abs(z[k] - ref[k]) for m, z in runs.items() if m != "ref"])
        rep[f"envelope_abs_{k}_per_iter"] = devs.max(0).tolist()
    path = os.path.join(HERE, "repro_floor_300.json")
    allrep = json.load(open(path)) if os.path.exists(path) else {}
    allrep[kind] = rep
    json.dump(allrep, open(path, "w"), indent=1)
    keep = np.arange(KEEP_EVERY - 1, TS, KEEP_EVERY)
    G.save(f"loop_{kind}_300", reg=np.array(r["reg"]), v_true=ref["v_true"], mu0=ref["mu0"],
           models=ref["models"][keep], keep=keep + 1, mu=ref["models"][-1][None, None],
           y_checksum=np.array([float(np.abs(ref["y"]).astype(np.float64).sum())]),
           params=np.array([TS, r["lr"], r["lam"], r["sigma"], 0, 0.0]), noise_type=np.array("gaussian"),
           sigma_x0=np.array(1e-4), use_time_weight=np.array(False), draw_rows=ref["draws"],
           env_model_rmse=env, **{"env_abs_" + k: np.array(rep[f"envelope_abs_{k}_per_iter"]) for k in metrics},
           **{k: ref[k] for k in ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")},
           **G.ctx_arrays(CTX))
    print(json.dumps({k: v for k, v in rep.items() if not k.endswith("per_iter")}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "member":
        torch.set_num_threads(int(os.environ.get("THREADS", "8")))
        run_member(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "combine":
        combine(sys.argv[2])
