"""Whole-loop parity of the drop-in InversionEngine on the HIP path against the reference's own
runs, with the reference's RNG draws replayed (tests/conftest.py:replay_draws):

* RED-DiffEq (regularization='diffusion', inversion.py:71-92, regularization/diffusion.py:50-83):
  eps_x0 -> t -> eps per iteration, the dim-8 U-Net of tests/golden/unet_dim8.npz, OpenFWI CurveVel
  (configs[2]'s loop) and the Marmousi 70x190 model whose regulariser takes the patched path
  (3 width-wise windows, diffusion.py:85-155; 310x430 padded grid);
* Gaussian noise + missing receivers with TV, Laplace noise + missing receivers with Tikhonov,
  B = 2 models (utils/data_trans.py:33-62,110-153);
* a 30-iteration TV trajectory against the reference's measured reproducibility floor
  (tests/golden/repro_floor.py).

Bar (BASELINE.md §4 / north_star): velocity-model RMSE vs the reference <= 1e-4 at the end of the
trajectory, per-iteration losses and metrics within fp32 tolerance.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ctx_of, load_golden, record_margin, replay_draws

pytestmark = pytest.mark.gpu


def make_fwi(ctx):
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
    return FWIForward(dict(ctx), "cuda", normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)


def dim8_diffusion(cuda):
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    z = load_golden("unet_dim8")
    net = Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1)
    net.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")})
    return GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                             objective="pred_noise").to(cuda).eval()


def run_engine(cuda, z, fwi=None, trace=None, repromote_after=None):
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.utils.ssim import SSIM
    if fwi is None:
        fwi = make_fwi(ctx_of(z))
    ts, lr, lam, sigma, missing, noise_std = z["params"]
    reg = str(z["reg"])
    reg = None if reg == "none" else reg
    if reg == "diffusion":
        dm = dim8_diffusion(cuda)
    else:
        class dm:
            device = cuda
    eng = InversionEngine(dm, SSIM(window_size=11), reg, use_time_weight=bool(z["use_time_weight"]),
                          sigma_x0=float(z["sigma_x0"]), show_progress=False)
    eng.model_trace = trace
    if repromote_after is not None:
        eng.repromote_after = repromote_after
    with replay_draws(z):
        mu, hist = eng.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]),
                                torch.from_numpy(z["y"]).to(cuda), fwi, ts=int(ts), lr=float(lr),
                                reg_lambda=float(lam), missing_number=int(missing), noise_std=float(noise_std),
                                noise_type=str(z["noise_type"]), regularization=reg)
    return mu.detach().cpu().numpy(), hist


def model_rmse(a, b):
    return np.sqrt(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2, axis=(1, 2, 3)))


@pytest.mark.parametrize("name", ["loop_red_openfwi", "loop_red_marmousi", "loop_noise_small", "loop_laplace_small"])
def test_loop_vs_reference_with_recorded_draws(cuda, name):
    z = load_golden(name)
    mu, hist = run_engine(cuda, z)
    d = model_rmse(mu, z["mu"])
    print(f"{name}: velocity-model RMSE vs the reference per model {d}")
    record_margin("loop_with_draws_model_rmse_vs_ref", name, float(d.max()), 1e-4)
    assert d.max() <= 1e-4, d                       # north_star: velocity-model RMSE within 1e-4
    for k in ("total_losses", "obs_losses", "reg_losses", "mae", "rmse", "ssim"):
        ref = np.atleast_2d(z[k]).astype(np.float64)
        got = np.array([h[k] for h in hist], np.float64)
        np.testing.assert_allclose(got, ref, rtol=2e-4, atol=1e-6, err_msg=k)


def test_red_loop_configs2_at_its_size(cuda):
    """configs[2]'s loop at its own size: OpenFWI CurveVel-A, 32 shots, nt = 1000, the dim-64 U-Net
    (synthetic weights, tests/golden/ckpt_weights.py), lambda 0.75, 3 iterations, the reference's
    eps_x0 / t / eps draws replayed.  Reference side: the reference engine, regulariser and U-Net
    driven by the oracle operator (the reference operator's autograd tape at this size is ~160 GB;
    make_golden.gen_loop_red_configs2).  The HIP forward regenerates y (its checksum pinned)."""
    import sys
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    from ckpt_weights import synth_param
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    from red_diffeq.utils.data_trans import v_normalize
    from red_diffeq.utils.ssim import SSIM
    z = load_golden("loop_red_configs2")
    fwi = make_fwi(ctx_of(z))
    with torch.no_grad():
        y = fwi(v_normalize(torch.from_numpy(z["v_true"])).to(cuda))
    ysum = float(y.abs().double().sum())
    assert abs(ysum - float(z["y_checksum"][0])) <= 1e-9 * ysum, (ysum, z["y_checksum"])
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
    diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250, objective="pred_noise")
    sd = diff.state_dict()
    diff.load_state_dict({k: (torch.from_numpy(synth_param(k, v.shape)) if k.startswith("model.") else v)
                          for k, v in sd.items()})
    diff = diff.to(cuda).eval()
    eng = InversionEngine(diff, SSIM(window_size=11), "diffusion", sigma_x0=1e-4, show_progress=False)
    with replay_draws(z):
        mu, hist = eng.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]), y, fwi, ts=3, lr=0.03,
                                reg_lambda=0.75, regularization="diffusion")
    d = float(model_rmse(mu.detach().cpu().numpy(), z["mu"])[0])
    print(f"loop_red_configs2: velocity-model RMSE vs the reference engine {d:.3e}")
    record_margin("loop_red_configs2_model_rmse_vs_ref", "", d, 1e-4)
    assert d <= 1e-4, d                               # north_star: velocity-model RMSE within 1e-4
    for k in ("total_losses", "obs_losses", "reg_losses", "mae", "rmse", "ssim"):
        np.testing.assert_allclose(np.array(hist[0][k], np.float64), z[k].astype(np.float64), rtol=2e-4, atol=1e-6,
                                   err_msg=k)


SSIM_B25_BAR = 2 * 1.85e-4   # 2 x K12's SSIM vs the reference's own on its final models (profiles/r5)


@pytest.mark.parametrize("adjoint", ["exact", "default"])
def test_red_loop_openfwi_yaml_b25(cuda, adjoint):
    """The reference's shipped OpenFWI config at its own batch (configs/openfwi/red-diffeq.yaml:43,
    batch_size 25: one optimize call on 25 CurveFault models x 5 shots with a B = 25 U-Net regulariser,
    reference inversion.py:46-129), nt = 400, the dim-8 U-Net, lambda 0.75, 3 iterations, the reference's
    eps_x0 / t / eps draws replayed.  Reference side: the reference engine, regulariser and U-Net driven
    by the oracle operator (make_golden.gen_loop_red_b25).  On the HIP side the 125 slices run as
    persistent launches of slice groups that span models.  Bar: model RMSE <= 1e-4 for every one of the
    25 models; losses and metrics within 2e-4 relative with the exact-order adjoint (gA bitwise the
    oracle's: only the U-Net's fp32 rounding differs); the default recurrence adjoint (dL/dv within ~1e-5
    of the exact gradient) within 5e-4 -- the reference engine on the oracle's FMA build, another correct
    fp32 operator (make_golden loop_red_b25_fma), is 7.9e-3 model RMSE and 2.6e-3 in SSIM away.
    SSIM's own floor is measured here: the metric (K12, its SSIM map in fp64) of the reference's OWN final
    25 models against the reference's value for them differs by ~1.9e-4 (the reference evaluates the
    variances E[x^2] - mu^2 in fp32; a GPU torch run of the reference SSIM module on the same models
    differs from it by 1.5e-4), so SSIM is held to a fixed 3.7e-4 = 2 x the committed floor
    (profiles/r5/ssim_metric_floor_b25.txt), and the floor itself is re-measured and held below 2e-4."""
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.utils.data_trans import v_normalize
    from red_diffeq.utils.ssim import SSIM
    z = load_golden("loop_red_b25")
    fwi = make_fwi(ctx_of(z))
    with torch.no_grad():
        y = fwi(v_normalize(torch.from_numpy(z["v_true"])).to(cuda))
    ysum = float(y.abs().double().sum())
    assert abs(ysum - float(z["y_checksum"][0])) <= 1e-9 * ysum, (ysum, z["y_checksum"])
    plan = fwi._plan(70, 70, y.device)
    assert plan.launch_info(25)["fwd_persistent"]
    plan.set_variant(adj_exact=adjoint == "exact")
    eng = InversionEngine(dim8_diffusion(cuda), SSIM(window_size=11), "diffusion", sigma_x0=1e-4,
                          show_progress=False)
    with replay_draws(z):
        mu, hist = eng.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]), y, fwi, ts=3, lr=0.03,
                                reg_lambda=0.75, regularization="diffusion")
    d = model_rmse(mu.detach().cpu().numpy(), z["mu"])
    print(f"loop_red_b25: velocity-model RMSE vs the reference engine per model: max {d.max():.3e}, median "
          f"{np.median(d):.3e}")
    record_margin("loop_red_b25_model_rmse_vs_ref", adjoint, float(d.max()), 1e-4)
    assert d.shape == (25,) and d.max() <= 1e-4, d
    from red_diffeq.core.fused import metrics
    with torch.no_grad():     # the metric's own floor: the reference's final models through K12
        m_ref = metrics(torch.from_numpy(z["mu"]).to(cuda).contiguous(),
                        v_normalize(torch.from_numpy(z["v_true"]).to(cuda)).contiguous()).cpu().numpy()
    floor = float(np.max(np.abs(m_ref[2] - z["ssim"][:, -1]) / np.abs(z["ssim"][:, -1])))
    # the floor measured here must stay the committed one (profiles/r5/ssim_metric_floor_b25.txt:
    # 1.85e-4): the SSIM bar below is a constant, so a drift of the metric cannot loosen it
    record_margin("loop_red_b25_ssim_metric_floor", "K12 on the reference's final models", floor, 2.0e-4)
    assert floor < 2.0e-4
    bar = 2e-4 if adjoint == "exact" else 5e-4
    for k in ("total_losses", "obs_losses", "reg_losses", "mae", "rmse", "ssim"):
        got = np.array([h[k] for h in hist], np.float64)
        ref = z[k].astype(np.float64)
        rel = float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-6)))
        # SSIM: K12 (its map in fp64, a deliberate departure from the reference's fp32 E[x^2] - mu^2)
        # differs from the reference's own value on identical models by 1.85e-4 (committed floor):
        # a fixed bar of 2 x that, 3.7e-4
        b = max(bar, SSIM_B25_BAR) if k == "ssim" else bar
        print(f"  {adjoint} {k}: max rel {rel:.3e} (bar {b:.2e})")
        record_margin("loop_red_b25_rel_" + adjoint, k, rel, b)
        # the assertion's own criterion |d| <= atol + b |ref|, as a fraction of its right-hand side
        record_margin("loop_red_b25_crit_" + adjoint, k, float(np.max(np.abs(got - ref) / (1e-6 + b * np.abs(ref)))), 1.0)
        np.testing.assert_allclose(got, ref, rtol=b, atol=1e-6, err_msg=k)


def test_engine_calls_a_non_reference_ssim_module(cuda):
    """with ssim_loss = SSIM(window_size=7) the engine's SSIM history is the caller's
    module evaluated on each iteration's model as the reference's MetricsCalculator does (reference
    core/inversion.py:55,94, core/metrics.py:13-46): equal, bit for bit, to MetricsCalculator(SSIM(7))
    on the traced models; with the reference's SSIM(11) the same run reports K12's (different) values,
    and MAE / RMSE / the losses are unchanged."""
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.core.metrics import MetricsCalculator
    from red_diffeq.utils.ssim import SSIM
    z = load_golden("loop_tv_openfwi")
    fwi = make_fwi(ctx_of(z))

    class _NoDiffusion:
        device = cuda

    runs = {}
    for w in (7, 11):
        eng = InversionEngine(_NoDiffusion(), SSIM(window_size=w), "tv", show_progress=False)
        eng.model_trace = []
        mu, hist = eng.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]),
                                torch.from_numpy(z["y"]).to(cuda), fwi, ts=4, lr=0.03, reg_lambda=0.01,
                                regularization="tv")
        runs[w] = (hist, eng.model_trace)
    hist7, trace7 = runs[7]
    calc = MetricsCalculator(SSIM(window_size=7))
    mu_true = torch.from_numpy(z["v_true"]).float().to(cuda)
    for it, m in enumerate(trace7):
        mae, rmse, ssim = calc.calculate(m, mu_true)
        for b in range(m.shape[0]):
            assert np.float32(hist7[b]["ssim"][it]) == np.float32(float(ssim[b])), (it, b)
            assert np.float32(hist7[b]["mae"][it]) == np.float32(float(mae[b]))
            assert np.float32(hist7[b]["rmse"][it]) == np.float32(float(rmse[b]))
    hist11 = runs[11][0]
    for k in ("total_losses", "obs_losses", "reg_losses"):
        assert np.array_equal(np.array(hist7[0][k]), np.array(hist11[0][k])), k
    np.testing.assert_allclose(np.array(hist7[0]["mae"]), np.array(hist11[0]["mae"]), rtol=1e-5)
    assert np.abs(np.array(hist7[0]["ssim"]) - np.array(hist11[0]["ssim"])).max() > 1e-4


def test_tv_long_trajectory_floor(cuda):
    """30 TV iterations: the HIP engine's model vs the reference's, per iteration, against the
    reference's own drift between 1 and 8 threads (measured: 0, bitwise) and between its operator and
    the oracle's (measured: 3.1e-4 after 30 iterations, 3.6e-4 peak; tests/golden/repro_floor.json).
    The final model is held to max(1e-4, 2 x that floor): the floor is one sample of a
    chaotic drift (another correct operator lands elsewhere in the same range)."""
    z = load_golden("loop_tv_long")
    mu, hist = run_engine(cuda, _with_defaults(z))
    rep = json.load(open(os.path.join(GOLDEN, "repro_floor.json")))
    floor = max(rep["final_ref8_vs_ref1"], rep["final_ref_vs_oracle_op"])
    d = float(model_rmse(mu, z["mu"])[0])
    print(f"loop_tv_long: velocity-model RMSE vs the reference {d:.3e} (oracle-operator floor {floor:.3e})")
    record_margin("loop_tv_long_model_rmse_vs_ref", "", d, max(1e-4, 2.0 * floor))
    assert d <= max(1e-4, 2.0 * floor), (d, floor)
    np.testing.assert_allclose(np.array(hist[0]["rmse"], np.float64), z["rmse"].astype(np.float64), atol=1e-4)


def _widen(env, w=25):
    """The ensemble's per-iteration deviation envelope widened by +-w iterations: the trajectories
    are chaotic (a sign flip moves a cell by +-lr), so when a divergence sets in differs between
    members by tens of iterations; a pointwise max over five members would flag the timing."""
    env = np.asarray(env, np.float64)
    return np.array([env[max(0, i - w):i + w + 1].max() for i in range(len(env))])


def _evidence(name, rec):
    """Append a measured-numbers record to $RDQ_EVIDENCE_DIR/<name>.jsonl (GPU evidence runs)."""
    d = os.environ.get("RDQ_EVIDENCE_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")


@pytest.mark.parametrize("adjoint", ["recurrence", "exact"])
@pytest.mark.parametrize("kind", ["tv", "red"])
def test_trajectory_300_within_ensemble(cuda, kind, adjoint):
    """The reference's full trajectory length (ts = 300, inversion.py:27 / default.yaml:35): TV
    (FlatVel-A) and RED-DiffEq (CurveVel-A, dim-8 U-Net, the reference's draws regenerated and
    replayed), ns = 2, nt = 1000, with both persistent adjoints (the default recurrence form and the
    exact-order one).  Bar: at every stored iteration (10, 20, ..., 300) the HIP model's RMSE vs the
    reference's is within max(1e-4, 2 x E_k), where E_k is the largest RMSE vs the reference of the
    five other correct fp32 operators driving the reference engine (tests/golden/make_long.py: the
    oracle, its FMA build, per-shot gradients, two extra-rounding runs) over iterations k +- 25
    (_widen: the trajectories are chaotic, divergence onsets differ by tens of iterations); the 2
    covers a sample max of five (leave-one-out over the members, 4-member envelopes: model <= 0.58,
    histories <= 1.05 of the bar).  MAE / RMSE / SSIM / misfit: the same rule on their deviations.
    North-star terms: the reference's own trajectory is reproducible only to E_k (~6e-3 model RMSE
    at ts = 300); the 1e-4 bar applies where E_k is below it."""
    z = _with_defaults(load_golden(f"loop_{kind}_300"))
    fwi = make_fwi(ctx_of(z))
    from red_diffeq.utils.data_trans import v_normalize
    with torch.no_grad():
        y = fwi(v_normalize(torch.from_numpy(z["v_true"])).to(cuda))
    ysum = float(y.abs().double().sum())
    assert abs(ysum - float(z["y_checksum"][0])) <= 1e-9 * ysum, (ysum, z["y_checksum"])
    fwi._plan(70, 70, cuda).set_variant(adj_exact=(adjoint == "exact"))
    z["y"] = y.cpu().numpy()
    trace = []
    mu, hist = run_engine(cuda, z, fwi, trace=trace)
    keep = z["keep"].astype(int)
    models = torch.stack(trace).cpu().numpy()[keep - 1, :, 0]          # (n_keep, B=1, 70, 70)
    d = model_rmse(models[:, 0:1], z["models"][:, None])
    env = _widen(z["env_model_rmse"])[keep - 1]
    bar = np.maximum(1e-4, 2.0 * env)
    rec = {"test": f"trajectory_300[{kind},{adjoint}]", "final_model_rmse_vs_ref": float(d[-1]),
           "max_model_rmse_vs_ref": float(d.max()), "ensemble_final": float(env[-1]),
           "ensemble_max": float(env.max()), "worst_ratio_to_bar": float((d / bar).max()),
           "model_rmse_vs_ref_at": {int(k): float(v) for k, v in zip(keep, d)}}
    for k in ("mae", "rmse", "ssim", "obs_losses"):
        got = np.array(hist[0][k], np.float64)
        dev = np.abs(got - z[k].astype(np.float64))
        lim = np.maximum(1e-6 if k != "obs_losses" else 1e-4 * np.abs(z[k]).max(), 2.0 * _widen(z["env_abs_" + k]))
        rec[f"{k}_max_abs_dev"] = float(dev.max())
        rec[f"{k}_worst_ratio_to_bar"] = float((dev / lim).max())
        rec[f"{k}_worst_iter"] = int(np.argmax(dev / lim)) + 1
    # before the chaotic divergence: iterations <= 50 against the ensemble's own pointwise
    # envelope, neither widened over +-25 iterations nor doubled (a systematic 1e-3-level kernel error
    # would show here; measured <= 0.96 of this bar, profiles/r3/trajectory_300.jsonl)
    early = keep <= 50
    early_bar = np.maximum(1e-4, np.asarray(z["env_model_rmse"], np.float64)[keep - 1])
    rec["early_worst_ratio_to_unwidened_envelope"] = float((d[early] / early_bar[early]).max())
    print(json.dumps(rec))
    _evidence("trajectory_300", rec)
    record_margin("trajectory_300_model_rmse_over_bar", f"{kind},{adjoint}", rec["worst_ratio_to_bar"], 1.0)
    record_margin("trajectory_300_early_over_unwidened_envelope", f"{kind},{adjoint}",
                  rec["early_worst_ratio_to_unwidened_envelope"], 1.0)
    assert np.all(d[early] <= early_bar[early]), list(zip(keep[early], d[early], early_bar[early]))
    assert np.all(d <= bar), list(zip(keep, d, bar))
    assert np.array_equal(models[-1, 0], mu[0, 0])
    for k in ("mae", "rmse", "ssim", "obs_losses"):
        assert rec[f"{k}_worst_ratio_to_bar"] <= 1.0, (k, rec)


class _with_defaults(dict):
    """npz view with the loop keys the round-1 fixtures do not carry."""

    def __init__(self, z):
        super().__init__({k: z[k] for k in z.files})
        self.setdefault("use_time_weight", np.array(False))
        self.setdefault("sigma_x0", np.array(1e-4))
        self.setdefault("noise_type", np.array("gaussian"))
        self.files = list(self.keys())

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        self.files = list(self.keys())


def test_persistent_failure_caught_inside_the_loop(cuda):
    """A persistent launch that cannot be resident (rdq_fwi_set_persistent(-1): grid oversubscribed
    2x past capacity, so the arrival barrier gives up and sets the status word) must never feed
    Adam: the fused step is guarded on the device, the engine sees the word within two iterations,
    rewinds to the failed iteration and replays on the chunked kernels.  The result is bitwise the
    run that used the chunked kernels from the start, and within the fixture's measured floor of
    the reference (tests/golden/repro_floor.json)."""
    z = _with_defaults(load_golden("loop_tv_openfwi"))
    fa = make_fwi(ctx_of(z))
    fa._plan(70, 70, cuda).set_persistent(False)
    mu_a, h_a = run_engine(cuda, z, fa)
    fb = make_fwi(ctx_of(z))
    pb = fb._plan(70, 70, cuda)
    pb.set_persistent(-1)
    with pytest.warns(RuntimeWarning, match="persistent FWI launch failed at iteration 0"):
        mu_b, h_b = run_engine(cuda, z, fb)
    assert not pb.launch_info(1)["fwd_persistent"]      # fell back to the chunked kernels
    assert np.array_equal(mu_a, mu_b)
    for k in h_a[0]:
        assert np.array_equal(np.array(h_a[0][k]), np.array(h_b[0][k])), k
    floor = json.load(open(os.path.join(GOLDEN, "repro_floor.json")))["oracle_op_floor_per_fixture"]
    assert float(model_rmse(mu_b, z["mu"])[0]) <= max(1e-4, 2.0 * floor["loop_tv_openfwi"])
    fb.check()                                          # status word cleared by the recovery


class _Switching:
    """The operator with its plan's persistent mode switched at given call numbers ({call: mode});
    forwards the fault-monitor interface of FWIForward (status_word / check / fallback / restore)."""

    def __init__(self, fwi, plan, at):
        self.fwi, self.plan, self.at, self.n = fwi, plan, dict(at), 0

    def to(self, device):
        return self

    def __call__(self, v):
        if self.n in self.at:
            self.plan.set_persistent(self.at[self.n])
        self.n += 1
        return self.fwi(v)

    def __getattr__(self, name):
        if name in ("status_word", "check", "fallback_to_chunked", "restore_persistent"):
            return getattr(self.fwi, name)
        raise AttributeError(name)


def test_persistent_failure_repromoted(cuda):
    """After a failed persistent launch the engine replays on the chunked kernels and, after
    repromote_after clean iterations, goes back to the persistent kernels: a fault at iteration 0
    with repromote_after = 2 equals (bitwise) a run on the chunked kernels for iterations 0-1 and the
    persistent ones from iteration 2."""
    z = _with_defaults(load_golden("loop_tv_openfwi"))
    fa = make_fwi(ctx_of(z))
    pa = fa._plan(70, 70, cuda)
    mu_a, h_a = run_engine(cuda, z, _Switching(fa, pa, {0: False, 2: True}))
    fb = make_fwi(ctx_of(z))
    pb = fb._plan(70, 70, cuda)
    pb.set_persistent(-1)
    with pytest.warns(RuntimeWarning, match="persistent FWI launch failed at iteration 0"):
        mu_b, h_b = run_engine(cuda, z, fb, repromote_after=2)
    assert pb.launch_info(1)["fwd_persistent"]          # re-promoted
    assert np.array_equal(mu_a, mu_b)
    for k in h_a[0]:
        assert np.array_equal(np.array(h_a[0][k]), np.array(h_b[0][k])), k
    fb.check()


def test_persistent_failure_mid_run_diffusion(cuda):
    """A persistent launch failing at iteration 4 of a RED-DiffEq run (U-Net on the side stream,
    iterations still queued when the fault is seen): the rewind restores the device RNG state, so
    the replayed iterations draw the same eps_x0 / t / eps from the device generator, and the result
    equals (bitwise) a run that switched to the chunked kernels at iteration 4 by itself."""
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.utils.ssim import SSIM
    z = load_golden("loop_red_openfwi")
    ts = 8

    def run(at):
        fwi = make_fwi(ctx_of(z))
        op = _Switching(fwi, fwi._plan(70, 70, cuda), at)
        eng = InversionEngine(dim8_diffusion(cuda), SSIM(window_size=11), "diffusion", sigma_x0=1e-4,
                              show_progress=False)
        eng.repromote_after = ts
        torch.manual_seed(77)
        mu, hist = eng.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]),
                                torch.from_numpy(z["y"]).to(cuda), op, ts=ts, lr=0.03, reg_lambda=0.75,
                                regularization="diffusion")
        return mu.detach().cpu().numpy(), hist, op.plan

    mu_a, h_a, _ = run({4: False})
    with pytest.warns(RuntimeWarning, match="persistent FWI launch failed at iteration 4"):
        mu_b, h_b, pb = run({4: -1})
    assert not pb.launch_info(1)["fwd_persistent"]
    assert np.array_equal(mu_a, mu_b)
    for k in h_a[0]:
        assert np.array_equal(np.array(h_a[0][k]), np.array(h_b[0][k])), k


def test_metrics_vs_reference_calculator(cuda):
    """K12 fused MAE / RMSE / SSIM vs the reference MetricsCalculator outputs
    (core/metrics.py:13-46; tests/golden/small_losses.npz m_mae / m_rmse / m_ssim)."""
    from red_diffeq.core.fused import metrics
    from red_diffeq.utils.data_trans import v_normalize
    z = load_golden("small_losses")
    b = torch.from_numpy(z["b"]).to(cuda)
    vtrue = (torch.from_numpy(z["c"]) + 1) / 2 * 3000 + 1500
    out = metrics(b, v_normalize(vtrue.to(cuda)).contiguous()).cpu().numpy()
    np.testing.assert_allclose(out[0], z["m_mae"], rtol=1e-5)
    np.testing.assert_allclose(out[1], z["m_rmse"], rtol=1e-5)
    np.testing.assert_allclose(out[2], z["m_ssim"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("reg", ["tv", "diffusion"])
def test_loop_has_no_per_iteration_host_sync(cuda, reg):
    """InversionEngine.optimize enqueues its iterations without a host <-> device synchronisation:
    under torch.cuda.set_sync_debug_mode("warn"), ts = 2 and ts = 8 report the same synchronising
    calls (the setup's host-to-device copies and the one history read after the loop).  Indexing a
    device tensor with a Python list (the metric reorder removed in round 3) was one such call per
    iteration and held the next forward until the host caught up."""
    import warnings
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.utils.ssim import SSIM
    z = load_golden("loop_red_openfwi")
    fwi = make_fwi(ctx_of(z))
    eng = InversionEngine(dim8_diffusion(cuda), SSIM(window_size=11), reg, sigma_x0=1e-4, show_progress=False)
    mu0, vt = torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"])
    y = torch.from_numpy(z["y"]).to(cuda)

    def syncs(ts):
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            torch.cuda.set_sync_debug_mode("warn")
            try:
                eng.optimize(mu0, vt, y, fwi, ts=ts, lr=0.03, reg_lambda=0.75, regularization=reg)
            finally:
                torch.cuda.set_sync_debug_mode(0)
        return [f"{x.filename}:{x.lineno}" for x in w if "synchroniz" in str(x.message)]

    syncs(2)                      # warm-up (graph capture, plan creation)
    a, b = syncs(2), syncs(8)
    assert len(a) == len(b), (a, b)
