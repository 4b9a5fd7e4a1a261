#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/*.npz by running the REFERENCE implementation
(SimingShan/red-diffeq at /root/reference) on the CPU of this container.

Run:  python tests/golden/make_golden.py [name ...]

This script is the only code in the repository that executes the reference.  It never runs on the
GPU box (the reference does not exist there); the tests only read the .npz files it writes.
Every fixture stores its inputs next to the reference outputs, so a test needs nothing else.
"""
import copy
import importlib.util
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refimport import load_reference  # noqa: E402

_spec = importlib.util.spec_from_file_location(
    "_synthetic", os.path.join(HERE, "..", "..", "red-diffeq_amd", "red_diffeq", "utils", "synthetic.py"))
synthetic = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(synthetic)

ref = load_reference()
torch.set_num_threads(8)

OPENFWI = dict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=5)
SMALL = dict(n_grid=16, nt=160, dx=10.0, dt=0.001, nbc=8, f=15.0, sz=10, gz=10, ng=16, ns=3)


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


def vnorm(v):
    return ref.data_trans.v_normalize(v)


def make_fwi(ctx, **kw):
    return ref.pde.FWIForward(copy.deepcopy(ctx), "cpu", normalize=True,
                              v_denorm_func=ref.data_trans.v_denormalize,
                              s_norm_func=ref.data_trans.s_normalize_none, **kw)


def ctx_arrays(ctx):
    return {"ctx_" + k: np.asarray(v) for k, v in ctx.items()}


# ----------------------------------------------------------------------------------------------
def gen_geometry():
    """ricker (pde.py:26-36) and adj_sr (pde.py:54-59) known-answer vectors."""
    out = {}
    f = make_fwi(OPENFWI)
    for i, (fq, dt, nt) in enumerate([(15.0, 1e-3, 1000), (10.0, 2e-3, 600), (25.0, 1e-3, 200)]):
        out[f"ricker{i}_args"] = np.array([fq, dt, nt])
        out[f"ricker{i}"] = f.ricker(fq, dt, nt)
    cases = [(70, 1, 70, 1.0), (70, 5, 70, 1.0), (70, 8, 70, 1.0), (70, 32, 70, 1.0),
             (70, 256, 70, 1.0), (190, 5, 190, 1.0), (70, 5, 70, 0.5), (16, 3, 16, 1.0)]
    for i, (n_grid, ns, ng, ss) in enumerate(cases):
        ctx = dict(OPENFWI, n_grid=n_grid, ns=ns, ng=ng)
        fw = make_fwi(ctx, sample_spatial=ss)
        c = fw.ctx
        isx, isz, igx, igz = fw.adj_sr(c["sx"], c["sz"], c["gx"], c["gz"], c["dx"], c["nbc"])
        out[f"sr{i}_args"] = np.array([n_grid, ns, ng, ss])
        out[f"sr{i}_isx"] = isx
        out[f"sr{i}_igx"] = igx
        out[f"sr{i}_isz_igz"] = np.array([isz, igz])
    # explicit sx/gx in ctx (grid units, pde.py:18-23)
    ctx = dict(SMALL, sx=[0, 7.5, 15], gx=list(range(0, 16, 3)))
    fw = make_fwi(ctx)
    c = fw.ctx
    isx, isz, igx, igz = fw.adj_sr(c["sx"], c["sz"], c["gx"], c["gz"], c["dx"], c["nbc"])
    out["srx_isx"], out["srx_igx"], out["srx_isz_igz"] = isx, igx, np.array([isz, igz])
    save("geometry", **out)


def gen_damp():
    """get_Abc sponge field (pde.py:38-52) for a small and an OpenFWI padded model."""
    out = {}
    for tag, ctx, nz, nx in [("small", SMALL, 16, 16), ("openfwi", OPENFWI, 70, 70),
                             ("rect", dict(SMALL, n_grid=24), 16, 24)]:
        v = synthetic.make_model("curvefault", nz, nx, seed=11, batch=2)
        fw = make_fwi(ctx)
        vpad = torch.nn.functional.pad(torch.from_numpy(v), (ctx["nbc"],) * 4, mode="replicate")
        damp = fw.get_Abc(vpad, ctx["nbc"], ctx["dx"])
        out[tag + "_v"] = v
        out[tag + "_damp"] = damp.numpy()
        out[tag + "_nbc_dx"] = np.array([ctx["nbc"], ctx["dx"]])
    save("damp", **out)


def run_forward(ctx, v, **kw):
    fw = make_fwi(ctx, **kw)
    with torch.no_grad():
        return fw(torch.from_numpy(vnorm(v))).numpy()


def gen_forward():
    """Forward seismograms, FWIForward.forward (pde.py:88-93)."""
    v = synthetic.make_model("curvefault", 16, 16, seed=3, batch=2)
    save("fwd_small", v=v, seis=run_forward(SMALL, v), **ctx_arrays(SMALL))
    save("fwd_small_st3", v=v, seis=run_forward(SMALL, v, sample_temporal=3, sample_spatial=0.5),
         st=np.array(3), ss=np.array(0.5), **ctx_arrays(SMALL))
    ctx = dict(SMALL, n_grid=24, nbc=4, nt=200, ns=4, ng=24)   # small sponge: periodic wrap matters
    v = synthetic.make_model("curvevel", 12, 24, seed=5, batch=1)
    save("fwd_wrap", v=v, seis=run_forward(ctx, v), **ctx_arrays(ctx))
    v = synthetic.make_model("flatvel", 70, 70, seed=8888, batch=1)
    ctx = dict(OPENFWI, ns=1)
    t0 = time.time()
    save("fwd_openfwi_ns1", v=v, seis=run_forward(ctx, v), **ctx_arrays(ctx))
    print(f"  openfwi ns1 forward {time.time() - t0:.1f}s")
    v = synthetic.make_model("curvevel", 70, 70, seed=8889, batch=1)
    ctx = dict(OPENFWI, ns=5, nt=400)
    save("fwd_openfwi_ns5_nt400", v=v, seis=run_forward(ctx, v), **ctx_arrays(ctx))


def l1_grad(ctx, v_true, v_init, mask=None):
    """Gradient of the reference observation loss (losses.py:14-41) through the autograd adjoint."""
    y = torch.from_numpy(run_forward(ctx, v_true))
    fw = make_fwi(ctx)
    vn = torch.from_numpy(vnorm(v_init)).clone().requires_grad_(True)
    pred = fw(vn)
    lc = ref.losses.LossCalculator(None)
    m = None if mask is None else torch.from_numpy(mask)
    loss = lc.observation_loss(pred, y, mask=m)
    loss.sum().backward()
    return y.numpy(), loss.detach().numpy(), vn.grad.numpy()


def smooth(v, sigma):
    from scipy.ndimage import gaussian_filter
    vn = gaussian_filter(vnorm(v.astype(np.float64)), sigma=sigma)
    return ref.data_trans.v_denormalize(vn).astype(np.float32)


def gen_grad():
    v_true = synthetic.make_model("curvefault", 16, 16, seed=21, batch=2)
    v_init = smooth(v_true, 2.0)
    y, loss, g = l1_grad(SMALL, v_true, v_init)
    save("grad_small", v_true=v_true, v_init=v_init, y=y, loss=loss, grad=g, **ctx_arrays(SMALL))
    mask = np.ones_like(y)
    mask[0, :, :, [2, 9]] = 0
    mask[1, :, :, [0, 5, 15]] = 0
    y, loss, g = l1_grad(SMALL, v_true, v_init, mask=mask)
    save("grad_small_mask", v_true=v_true, v_init=v_init, y=y, mask=mask, loss=loss, grad=g,
         **ctx_arrays(SMALL))
    # flat layers: many ties for vmin (torch.min first-index rule), OpenFWI geometry, ns=1
    v_true = synthetic.make_model("flatvel", 70, 70, seed=8888, batch=1)
    v_init = smooth(v_true, 10.0)
    v_init[0, 0, 0:3, :] = v_init.min()   # force ties for the minimum in the top rows
    ctx = dict(OPENFWI, ns=1)
    t0 = time.time()
    y, loss, g = l1_grad(ctx, v_true, v_init)
    print(f"  openfwi ns1 fwd+adj {time.time() - t0:.1f}s")
    save("grad_openfwi_ns1", v_true=v_true, v_init=v_init, y=y, loss=loss, grad=g, **ctx_arrays(ctx))


class _NoDiffusion:
    device = torch.device("cpu")


RNG_FNS = ("randn", "rand", "randint", "randperm")


class record_draws:
    """Record every draw the reference makes from torch's global RNG (torch.randn / rand / randint /
    randperm with generator=None), in call order.  The GPU tests replay them
    (tests/conftest.py:replay_draws): the device RNG stream differs from the CPU one, so injected
    draws are the only way to pin an RNG-driven trajectory (eps_x0 at inversion.py:73, t at
    regularization/diffusion.py:57, eps at :63, noise at utils/data_trans.py:55/59, missing
    receivers at :146)."""

    def __init__(self):
        self.kinds, self.vals = [], []

    def __enter__(self):
        self.orig = {n: getattr(torch, n) for n in RNG_FNS}
        for n in RNG_FNS:
            def wrap(*a, _n=n, **kw):
                assert kw.get("generator") is None, "only global-RNG draws are recorded"
                r = self.orig[_n](*a, **kw)
                self.kinds.append(_n)
                self.vals.append(r.detach().cpu().numpy().copy())
                return r
            setattr(torch, n, wrap)
        return self

    def __exit__(self, *exc):
        for n, f in self.orig.items():
            setattr(torch, n, f)

    def arrays(self):
        out = {"draw_kinds": np.array(self.kinds, dtype="U16")}
        out.update({f"draw{i}": v for i, v in enumerate(self.vals)})
        return out


def run_loop(ctx, family, seed, reg, ts, lr, lam, sigma, missing=0, noise_std=0.0, noise_type="gaussian",
             batch=1, nz=None, diffusion=None, sigma_x0=1e-4, use_time_weight=False, record=False):
    nz = nz or ctx["n_grid"]
    v_true = synthetic.make_model(family, nz, ctx["n_grid"], seed=seed, batch=batch)
    y = torch.from_numpy(run_forward(ctx, v_true))
    init = torch.cat([ref.data_trans.prepare_initial_model(torch.from_numpy(v_true[i:i + 1]), "smoothed",
                                                           sigma=sigma) for i in range(batch)])
    mu0 = torch.nn.functional.pad(init, (1, 1, 1, 1), "constant", 0)
    eng = ref.inversion.InversionEngine(diffusion if diffusion is not None else _NoDiffusion(),
                                        ref.ssim.SSIM(window_size=11), reg, use_time_weight=use_time_weight,
                                        sigma_x0=sigma_x0)
    torch.manual_seed(1234)
    rec = record_draws()
    with rec:
        mu, hist = eng.optimize(mu0, torch.from_numpy(v_true), y, make_fwi(ctx), ts=ts, lr=lr,
                                reg_lambda=lam, missing_number=missing, noise_std=noise_std,
                                noise_type=noise_type, regularization=reg)
    keys = ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")
    if batch == 1:      # round-1 layout: 1-D histories of model 0
        hs = {k: np.array(hist[0][k]) for k in keys}
    else:               # (B, ts)
        hs = {k: np.stack([np.array(h[k]) for h in hist]) for k in keys}
    out = dict(v_true=v_true, y=y.numpy(), mu0=mu0.numpy(), mu=mu.detach().numpy(),
               params=np.array([ts, lr, lam, sigma, missing, noise_std]), noise_type=np.array(noise_type),
               sigma_x0=np.array(sigma_x0), use_time_weight=np.array(use_time_weight), **hs, **ctx_arrays(ctx))
    if record:
        out.update(rec.arrays())
    return out


def gen_loop():
    """InversionEngine.optimize trajectories (inversion.py:26-129), TV and Tikhonov."""
    t0 = time.time()
    ctx = dict(OPENFWI, ns=2)
    save("loop_tv_openfwi", reg=np.array("tv"),
         **run_loop(ctx, "flatvel", 8888, "tv", ts=5, lr=0.03, lam=0.01, sigma=10.0))
    print(f"  tv loop {time.time() - t0:.1f}s")
    ctx = dict(SMALL, n_grid=16)
    save("loop_l2_small", reg=np.array("l2"),
         **run_loop(ctx, "curvevel", 77, "l2", ts=8, lr=0.03, lam=0.1, sigma=2.0))
    save("loop_none_small", reg=np.array("none"),
         **run_loop(ctx, "curvevel", 78, None, ts=8, lr=0.05, lam=0.0, sigma=2.0))


def gen_loop_rng():
    """InversionEngine trajectories whose RNG draws are recorded for replay: Gaussian noise +
    missing receivers (TV) and Laplace noise + missing receivers (Tikhonov), B = 2 models (one
    randperm per model, the same receivers for every shot: data_trans.py:110-153)."""
    ctx = dict(SMALL, n_grid=16)
    for name, fam, seed, reg, lam, missing, std, kind in (
            ("loop_noise_small", "curvefault", 81, "tv", 0.05, 4, 0.05, "gaussian"),
            ("loop_laplace_small", "curvevel", 82, "l2", 0.1, 3, 0.02, "laplace")):
        out = run_loop(ctx, fam, seed, reg, ts=6, lr=0.03, lam=lam, sigma=2.0, missing=missing,
                       noise_std=std, noise_type=kind, batch=2, record=True)
        # the perturbed data and mask the engine built (its first draws after manual_seed(1234),
        # inversion.py:63-64), for the CPU test of the two helpers alone
        torch.manual_seed(1234)
        yn = ref.data_trans.add_noise_to_seismic(torch.from_numpy(out["y"]), std, noise_type=kind)
        yn, mask = ref.data_trans.missing_trace(yn, missing, return_mask=True)
        save(name, reg=np.array(reg), y_noisy=yn.numpy(), mask=mask.numpy(), **out)


def gen_loop_red():
    """RED-DiffEq loop (InversionEngine.optimize(regularization='diffusion'), inversion.py:71-92 +
    regularization/diffusion.py:50-83) with the dim-8 U-Net of gen_unet, its eps_x0 / t / eps draws
    recorded: OpenFWI CurveVel grid (configs[2]'s family and loop: lambda 0.75, lr 0.03,
    sigma_x0 1e-4), and the Marmousi 70x190 model (310x430 padded) whose regulariser runs the
    patched path (3 width-wise windows, diffusion.py:85-155), configs/marmousi/red-diffeq.yaml."""
    diff = ref.diffusion.GaussianDiffusion(_unet_dim8(), image_size=72, timesteps=1000, sampling_timesteps=250,
                                           objective="pred_noise").eval()
    t0 = time.time()
    ctx = dict(OPENFWI, ns=2)
    save("loop_red_openfwi", reg=np.array("diffusion"),
         **run_loop(ctx, "curvevel", 8890, "diffusion", ts=6, lr=0.03, lam=0.75, sigma=10.0,
                    diffusion=diff, record=True))
    print(f"  red openfwi loop {time.time() - t0:.1f}s")
    t0 = time.time()
    ctx = dict(OPENFWI, n_grid=190, ng=190, ns=2)
    save("loop_red_marmousi", reg=np.array("diffusion"),
         **run_loop(ctx, "curvefault", 8891, "diffusion", ts=3, lr=0.03, lam=0.75, sigma=20.0, nz=70,
                    diffusion=diff, record=True))
    print(f"  red marmousi loop {time.time() - t0:.1f}s")


class _OracleOp(torch.autograd.Function):
    @staticmethod
    def forward(c, v, f):
        seis, cf = f.forward(v.detach().contiguous().numpy().astype(np.float32), keep_history=True)
        c.f, c.cf = f, cf
        return torch.from_numpy(seis)

    @staticmethod
    def backward(c, g):
        gA, gK, gb = c.f.adjoint(c.cf, g.contiguous().numpy())
        out = torch.from_numpy(c.f.finalize(c.cf, gA, gK, gb))
        c.cf = None
        return out, None


class _OracleFWI:
    """The oracle (oracle/fwi_oracle.c, the kernels' summation order; forward bit-exact with the
    reference operator, gradient within 1e-5) as a differentiable operator for the reference engine."""

    def __init__(self, ctx):
        sys.path.insert(0, os.path.join(HERE, "..", ".."))
        from oracle import oracle as O
        self.f = O.OracleFWI(ctx, 1)

    def __call__(self, v):
        return _OracleOp.apply(v, self.f)

    def to(self, device):
        return self


def gen_loop_red_configs2():
    """configs[2]'s loop at its own size: OpenFWI CurveVel-A, 32 shots, nt = 1000, the reference
    architecture's dim-64 U-Net (weights tests/golden/ckpt_weights.py, default sigmoid schedule),
    lambda 0.75, lr 0.03, sigma_x0 1e-4, 3 iterations, the eps_x0 / t / eps draws recorded.  The
    reference FWIForward's autograd tape at 32 shots x 1000 steps is ~160 GB, so the reference engine,
    regulariser and U-Net are driven by the oracle operator (pinned to the reference operator at
    smaller sizes); y is the oracle forward (bit-exact with the reference's).  y (9 MB) is not stored:
    the GPU test regenerates it with the HIP forward, bit-exact with the oracle's."""
    from ckpt_weights import synth_param
    torch.manual_seed(0)
    net = ref.diffusion.Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1, flash_attn=False)
    diff = ref.diffusion.GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                                           objective="pred_noise")
    sd = diff.state_dict()
    diff.load_state_dict({k: (torch.from_numpy(synth_param(k, v.shape)) if k.startswith("model.") else v)
                          for k, v in sd.items()})
    diff.eval()
    ctx = dict(OPENFWI, ns=32)
    v_true = synthetic.make_model("curvevel", 70, 70, seed=8888, batch=1)
    op = _OracleFWI(ctx)
    with torch.no_grad():
        y = op.f.forward(vnorm(v_true).astype(np.float32))[0]
    init = ref.data_trans.prepare_initial_model(torch.from_numpy(v_true), "smoothed", sigma=10.0)
    mu0 = torch.nn.functional.pad(init, (1, 1, 1, 1), "constant", 0)
    eng = ref.inversion.InversionEngine(diff, ref.ssim.SSIM(window_size=11), "diffusion", sigma_x0=1e-4)
    ts = 3
    torch.manual_seed(1234)
    rec = record_draws()
    with rec:
        mu, hist = eng.optimize(mu0, torch.from_numpy(v_true), torch.from_numpy(y), op, ts=ts, lr=0.03,
                                reg_lambda=0.75, regularization="diffusion")
    keys = ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")
    save("loop_red_configs2", reg=np.array("diffusion"), v_true=v_true, mu0=mu0.numpy(), mu=mu.detach().numpy(),
         params=np.array([ts, 0.03, 0.75, 10.0, 0, 0.0]), noise_type=np.array("gaussian"), sigma_x0=np.array(1e-4),
         use_time_weight=np.array(False), y_checksum=np.array([float(np.abs(y).astype(np.float64).sum())]),
         **{k: np.array(hist[0][k]) for k in keys}, **ctx_arrays(ctx), **rec.arrays())


class _OracleOpPerModel(torch.autograd.Function):
    """The oracle operator one model at a time (B models x ns shots): the forward keeps no history and the
    backward recomputes each model's forward with its history before the adjoint, so at most one model's
    history (0.8 GB at ns = 5, nt = 400) is alive.  The oracle's arithmetic is per (model, shot), so this
    equals the batched oracle bit for bit."""

    @staticmethod
    def forward(c, v, f):
        vn = v.detach().contiguous().numpy().astype(np.float32)
        c.f, c.vn = f, vn
        return torch.from_numpy(np.concatenate([f.forward(vn[b:b + 1])[0] for b in range(vn.shape[0])]))

    @staticmethod
    def backward(c, g):
        g = g.contiguous().numpy()
        out = []
        for b in range(c.vn.shape[0]):
            _, cf = c.f.forward(c.vn[b:b + 1], keep_history=True)
            gA, gK, gb = c.f.adjoint(cf, g[b:b + 1])
            out.append(c.f.finalize(cf, gA, gK, gb))
            del cf
        return torch.from_numpy(np.concatenate(out)), None


def gen_loop_red_b25(variant=""):
    """The reference's shipped OpenFWI config at its own batch (configs/openfwi/red-diffeq.yaml:43,
    batch_size 25: one InversionEngine.optimize call on 25 models x 5 shots, inversion.py:46-129, with a
    B = 25 U-Net regulariser): 25 CurveFault models, nt = 400, the dim-8 U-Net of gen_unet, lambda 0.75,
    lr 0.03, sigma 10, sigma_x0 1e-4, 3 iterations, the eps_x0 / t / eps draws recorded.  The reference
    engine, regulariser and U-Net are driven by the oracle operator (one model at a time, recomputed in
    the backward: the reference FWIForward's autograd tape at 125 slices x 400 steps is ~25 GB).  y is the
    oracle forward (bit-exact with the reference operator's); it is not stored (14 MB): the GPU test
    regenerates it with the HIP forward and checks its checksum."""
    diff = ref.diffusion.GaussianDiffusion(_unet_dim8(), image_size=72, timesteps=1000, sampling_timesteps=250,
                                           objective="pred_noise").eval()
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from oracle import oracle as O
    ctx = dict(OPENFWI, nt=400)
    B = 25
    v_true = synthetic.make_model("curvefault", 70, 70, seed=8892, batch=B)
    f = O.OracleFWI(ctx, 1, variant=variant)
    vt = vnorm(v_true).astype(np.float32)
    y = np.concatenate([f.forward(vt[b:b + 1])[0] for b in range(B)])

    class Op:
        def __call__(self, v):
            return _OracleOpPerModel.apply(v, f)

        def to(self, device):
            return self
    init = torch.cat([ref.data_trans.prepare_initial_model(torch.from_numpy(v_true[i:i + 1]), "smoothed", sigma=10.0)
                      for i in range(B)])
    mu0 = torch.nn.functional.pad(init, (1, 1, 1, 1), "constant", 0)
    eng = ref.inversion.InversionEngine(diff, ref.ssim.SSIM(window_size=11), "diffusion", sigma_x0=1e-4)
    ts = 3
    torch.manual_seed(1234)
    rec = record_draws()
    t0 = time.time()
    with rec:
        mu, hist = eng.optimize(mu0, torch.from_numpy(v_true), torch.from_numpy(y), Op(), ts=ts, lr=0.03,
                                reg_lambda=0.75, regularization="diffusion")
    print(f"  b25 loop {time.time() - t0:.1f}s")
    keys = ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")
    if variant:      # reproducibility-floor member: the same engine and draws on another correct fp32 operator
        save("loop_red_b25_" + variant, mu=mu.detach().numpy(), **{k: np.stack([np.array(h[k]) for h in hist])
                                                                    for k in keys})
        return
    save("loop_red_b25", reg=np.array("diffusion"), v_true=v_true, mu0=mu0.numpy(), mu=mu.detach().numpy(),
         params=np.array([ts, 0.03, 0.75, 10.0, 0, 0.0]), noise_type=np.array("gaussian"), sigma_x0=np.array(1e-4),
         use_time_weight=np.array(False), y_checksum=np.array([float(np.abs(y).astype(np.float64).sum())]),
         **{k: np.stack([np.array(h[k]) for h in hist]) for k in keys}, **ctx_arrays(ctx), **rec.arrays())


def gen_initial():
    """prepare_initial_model (utils/data_trans.py:65-107), all three initial_type branches."""
    out = {}
    for i, (fam, nz, nx) in enumerate([("curvefault", 70, 70), ("flatvel", 70, 190)]):
        v = synthetic.make_model(fam, nz, nx, seed=40 + i, batch=1)
        out[f"v{i}"] = v
        out[f"v{i}_smoothed"] = ref.data_trans.prepare_initial_model(torch.from_numpy(v), "smoothed",
                                                                     sigma=10.0).numpy()
        out[f"v{i}_homogeneous"] = ref.data_trans.prepare_initial_model(torch.from_numpy(v), "homogeneous").numpy()
        out[f"v{i}_linear"] = ref.data_trans.prepare_initial_model(torch.from_numpy(v), "linear").numpy()
    save("initial_models", **out)


def gen_ckpt():
    """dim-64 checkpoint round trip (the reference architecture, 296 state_dict keys): weights from
    tests/golden/ckpt_weights.py, schedule buffers from a LINEAR beta schedule, loaded into the
    reference's default (sigmoid) GaussianDiffusion the way scripts/run_inversion.py:63-67 does, so
    the checkpoint's buffers override the computed ones.  Records eps-hat, pred_noise / pred_x_start
    of model_predictions(clip_x_start=True, rederive_pred_noise=True) for 2 inputs."""
    from ckpt_weights import synth_param
    torch.manual_seed(0)
    net = ref.diffusion.Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1, flash_attn=False)
    diff = ref.diffusion.GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                                           objective="pred_noise")
    lin = ref.diffusion.GaussianDiffusion(ref.diffusion.Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1),
                                          image_size=72, timesteps=1000, sampling_timesteps=250,
                                          objective="pred_noise", beta_schedule="linear")
    sd = diff.state_dict()
    new = {}
    bufs = {}
    for k, v in sd.items():
        if k.startswith("model."):
            new[k] = torch.from_numpy(synth_param(k, v.shape))
        else:
            new[k] = lin.state_dict()[k].clone()
            bufs["buf." + k] = new[k].numpy()
    diff.load_state_dict(new)
    diff.eval()
    g = torch.Generator().manual_seed(12)
    x = torch.randn(2, 1, 72, 72, generator=g).clamp(-3, 3)
    t = torch.tensor([40, 650])
    with torch.no_grad():
        eps = diff.model(x, t, None)
        pred = diff.model_predictions(x, t, x_self_cond=None, clip_x_start=True, rederive_pred_noise=True)
    save("ckpt_dim64", x=x.numpy(), t=t.numpy(), eps=eps.numpy(), pred_noise=pred.pred_noise.numpy(),
         pred_x_start=pred.pred_x_start.numpy(), keys=np.array(list(sd.keys())),
         shapes=np.array([list(v.shape) + [0] * (4 - v.dim()) for v in sd.values()]), **bufs)


def _unet_dim8(seed=0):
    torch.manual_seed(seed)
    net = ref.diffusion.Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1, flash_attn=False)
    # perturb the unit-initialised norm gains so that the fixture pins them
    with torch.no_grad():
        for name, p in net.named_parameters():
            if name.endswith(".g") or (".norm." in name and name.endswith("weight")):
                p.mul_(1.0 + 0.2 * torch.randn_like(p))
            if ".norm." in name and name.endswith("bias"):
                p.add_(0.1 * torch.randn_like(p))
    return net.eval()


def gen_unet():
    """lucidrains U-Net forward (models/diffusion.py:220-301) at dim=8, same topology."""
    net = _unet_dim8()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 1, 72, 72, generator=g)
    t = torch.tensor([17, 803])
    with torch.no_grad():
        out = net(x, t)
    sd = {"sd." + k: v.numpy() for k, v in net.state_dict().items()}
    save("unet_dim8", x=x.numpy(), t=t.numpy(), out=out.numpy(), **sd)


def gen_red():
    """RED-DiffEq regularizer (regularization/diffusion.py:50-155) + schedule buffers."""
    net = _unet_dim8()
    diff = ref.diffusion.GaussianDiffusion(net, image_size=72, timesteps=1000,
                                           sampling_timesteps=250, objective="pred_noise").eval()
    out = {"buf." + k: v.numpy() for k, v in diff.state_dict().items() if not k.startswith("model.")}
    for tag, H, W, tw in [("sq", 72, 72, False), ("sqw", 72, 72, True), ("patch", 72, 192, False)]:
        red = ref.reg_diffusion.RED_DiffEq(diff, use_time_weight=tw, sigma_x0=1e-4)
        g = torch.Generator().manual_seed(99)
        mu = (torch.rand(2, 1, H, W, generator=g) * 2 - 1).requires_grad_(True)
        seed = 4242
        gen = torch.Generator().manual_seed(seed)
        if W > 72:
            reg, gpm, t = red.get_reg_loss_patched(mu, generator=gen)
        else:
            reg, gpm, t = red.get_reg_loss(mu, generator=gen)
        reg.sum().backward()
        # replay the generator to record the injected draws (t first, then noise)
        gen = torch.Generator().manual_seed(seed)
        t2 = torch.randint(0, 1000, (2,), generator=gen, dtype=torch.long)
        shp = (2, 1, H - 2, W - 2) if W > 72 else (2, 1, H, W)
        noise = torch.randn(shp, generator=gen)
        assert torch.equal(t, t2)
        out.update({tag + "_mu": mu.detach().numpy(), tag + "_t": t.numpy(),
                    tag + "_noise": noise.numpy(), tag + "_reg": reg.detach().numpy(),
                    tag + "_gpm": gpm.detach().numpy(), tag + "_grad": mu.grad.numpy(),
                    tag + "_seed": np.array(seed)})
    save("red_dim8", **out)


def gen_small_losses():
    """TV / Tikhonov (regularization/benchmark.py:4-37), SSIM (utils/ssim.py), metrics."""
    g = torch.Generator().manual_seed(7)
    a = torch.rand(3, 1, 72, 72, generator=g) * 2 - 1
    b = torch.rand(3, 1, 70, 70, generator=g) * 2 - 1
    c = torch.rand(3, 1, 70, 70, generator=g) * 2 - 1
    s = ref.ssim.SSIM(window_size=11)
    ssim = np.array([s((b[i:i + 1] + 1) / 2, (c[i:i + 1] + 1) / 2).item() for i in range(3)])
    mc = ref.metrics.MetricsCalculator(ref.ssim.SSIM(window_size=11))
    vtrue = ref.data_trans.v_denormalize(c)
    mae, rmse, ss = mc.calculate(b, vtrue)
    save("small_losses", a=a.numpy(), b=b.numpy(), c=c.numpy(),
         tv=ref.reg_bench.total_variation_loss(a).numpy(),
         l2=ref.reg_bench.tikhonov_loss(a).numpy(), ssim=ssim,
         m_mae=mae.numpy(), m_rmse=rmse.numpy(), m_ssim=ss.numpy(),
         patches_190_70=np.array(ref.reg_diffusion.calculate_patches(190, 70)[0]),
         overlaps_190_70=np.array(ref.reg_diffusion.calculate_patches(190, 70)[1]))


def gen_dfwi():
    """DiffusionFWI baseline (diffusion_bench/diffusionfwi.py:79-366) on a 14x14 model (16x16 after
    diffusion_pad: U-Net-divisible), dim-8 U-Net of gen_unet, two variants: the defaults
    (grad_norm, grad_clip 1.0) and with grad_smooth 1.0.  No RNG draws (noise_std 0, no missing
    traces), so the trajectory is a pure function of the inputs."""
    spec = importlib.util.spec_from_file_location("_ref_dfwi", "/root/reference/diffusion_bench/diffusionfwi.py")
    dfwi = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(dfwi)
    ctx = dict(SMALL, n_grid=14, ng=14, ns=2)
    v_true = synthetic.make_model("curvefault", 14, 14, seed=31, batch=1)
    y = torch.from_numpy(run_forward(ctx, v_true))
    init = ref.data_trans.prepare_initial_model(torch.from_numpy(v_true), "smoothed", sigma=3.0)
    net = _unet_dim8()
    diff = ref.diffusion.GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                                           objective="pred_noise").eval()
    out = dict(v_true=v_true, y=y.numpy(), mu0=init.numpy(), **ctx_arrays(ctx))
    for tag, kw in (("base", {}), ("smooth", dict(grad_smooth=1.0))):
        fwi = make_fwi(ctx)
        bench = dfwi.DiffusionFWI(diff, fwi, ref.ssim.SSIM(window_size=11))
        mu, hist = bench.optimize(init.clone(), torch.from_numpy(v_true), y, fwi, ts=3, diffusion_ts=4, lr=0.03,
                                  **kw)
        h = hist[0]
        out.update({tag + "_mu": mu.detach().numpy(), tag + "_obs": np.array(h["obs_losses"]).ravel(),
                    tag + "_ssim": np.array(h["ssim"]).ravel(), tag + "_mae": np.array(h["mae"]).ravel(),
                    tag + "_rmse": np.array(h["rmse"]).ravel()})
    save("dfwi_small", **out)


def gen_ilvr():
    """ILVR_FWI (diffusion_bench/ilvr_fwi.py) on the gen_dfwi case with the q_sample noise drawn from a
    seeded generator and recorded (the draw is torch.randn_like inside _apply_ilvr), plus the
    Resizer (diffusion_bench/resizer.py) down/up outputs at the factors the schedule uses."""
    import types
    pkg = types.ModuleType("diffusion_bench")
    pkg.__path__ = ["/root/reference/diffusion_bench"]
    sys.modules["diffusion_bench"] = pkg
    ilvr = importlib.import_module("diffusion_bench.ilvr_fwi")
    rz = importlib.import_module("diffusion_bench.resizer")
    out = {}
    g = torch.Generator().manual_seed(17)
    x = torch.rand(2, 1, 70, 70, generator=g) * 2 - 1
    out["rz_x"] = x.numpy()
    for n in (16, 9, 5, 2):
        d = rz.Resizer(x.shape, 1 / n)(x)
        u = rz.Resizer((2, 1, int(70 / n), int(70 / n)), n)(d)
        out[f"rz_down{n}"], out[f"rz_up{n}"] = d.numpy(), u.numpy()
    ctx = dict(SMALL, n_grid=14, ng=14, ns=2)
    v_true = synthetic.make_model("curvefault", 14, 14, seed=31, batch=1)
    y = torch.from_numpy(run_forward(ctx, v_true))
    init = ref.data_trans.prepare_initial_model(torch.from_numpy(v_true), "smoothed", sigma=3.0)
    diff = ref.diffusion.GaussianDiffusion(_unet_dim8(), image_size=72, timesteps=1000, sampling_timesteps=250,
                                           objective="pred_noise").eval()
    draws = []
    gen = torch.Generator().manual_seed(23)
    orig = torch.randn_like

    def seeded_randn_like(t, **kw):
        r = torch.randn(t.shape, generator=gen, dtype=t.dtype)
        draws.append(r.numpy().copy())
        return r

    torch.randn_like = seeded_randn_like
    try:
        fwi = make_fwi(ctx)
        bench = ilvr.ILVR_FWI(diff, fwi, ref.ssim.SSIM(window_size=11))
        mu, hist = bench.optimize(init.clone(), torch.from_numpy(v_true), y, fwi, ts=3, diffusion_ts=4, lr=0.03,
                                  ilvr_weight=0.3)
    finally:
        torch.randn_like = orig
    h = hist[0]
    out.update(v_true=v_true, y=y.numpy(), mu0=init.numpy(), noise=np.stack(draws), mu=mu.detach().numpy(),
               obs=np.array(h["obs_losses"]).ravel(), ssim=np.array(h["ssim"]).ravel(),
               mae=np.array(h["mae"]).ravel(), rmse=np.array(h["rmse"]).ravel(), **ctx_arrays(ctx))
    save("ilvr_small", **out)


def gen_post():
    """RED_DiffEq_POST_PROCESS.diffusion_denoise (regularization/diffusion.py:158-200) with the dim-8
    U-Net of gen_unet: q_sample to t = 6, then 6 p_sample_deterministic steps
    (models/diffusion.py:431-452); its randn_like draw from a seeded generator, recorded.  Also
    p_mean_variance / p_sample_deterministic alone at three timesteps."""
    diff = ref.diffusion.GaussianDiffusion(_unet_dim8(), image_size=72, timesteps=1000, sampling_timesteps=250,
                                           objective="pred_noise").eval()
    g = torch.Generator().manual_seed(31)
    mu = torch.rand(2, 1, 72, 72, generator=g) * 2 - 1
    x = torch.randn(2, 1, 72, 72, generator=g).clamp(-2, 2)
    out = {"mu": mu.numpy(), "x": x.numpy()}
    with torch.no_grad():
        for t in (0, 37, 640):
            mean, var, logvar, xs = diff.p_mean_variance(x, torch.full((2,), t, dtype=torch.long))
            out[f"pmv{t}_mean"], out[f"pmv{t}_xs"] = mean.numpy(), xs.numpy()
            out[f"pmv{t}_var"], out[f"pmv{t}_logvar"] = var.reshape(-1).numpy(), logvar.reshape(-1).numpy()
            m2, xs2 = diff.p_sample_deterministic(x, t)
            assert torch.equal(m2, mean) and torch.equal(xs2, xs)
    draws = []
    gen = torch.Generator().manual_seed(32)
    orig = torch.randn_like

    def seeded_randn_like(t, **kw):
        r = torch.randn(t.shape, generator=gen, dtype=t.dtype)
        draws.append(r.numpy().copy())
        return r
    torch.randn_like = seeded_randn_like
    try:
        with torch.no_grad():
            den = ref.reg_diffusion.RED_DiffEq_POST_PROCESS(diff).diffusion_denoise(mu, 6)
    finally:
        torch.randn_like = orig
    assert len(draws) == 1
    save("post_dim8", noise=draws[0], denoised=den.numpy(), timesteps=np.array(6), **out)


GENS = dict(geometry=gen_geometry, damp=gen_damp, forward=gen_forward, grad=gen_grad,
            loop=gen_loop, unet=gen_unet, red=gen_red, small_losses=gen_small_losses, dfwi=gen_dfwi,
            ilvr=gen_ilvr, loop_rng=gen_loop_rng, loop_red=gen_loop_red, initial=gen_initial, ckpt=gen_ckpt,
            loop_red_configs2=gen_loop_red_configs2, post=gen_post, loop_red_b25=gen_loop_red_b25,
            loop_red_b25_fma=lambda: gen_loop_red_b25("fma"))

if __name__ == "__main__":
    names = sys.argv[1:] or list(GENS)
    for n in names:
        t0 = time.time()
        GENS[n]()
        print(f"[{n}] {time.time() - t0:.1f}s")
