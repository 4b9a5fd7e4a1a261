"""Host-side logic on CPU: geometry, config, schedules, patching, the C-ABI library surface and
the no-CPU-fallback rule."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden


def test_ricker_and_geometry_vs_reference():
    from red_diffeq.solvers.pde import FWIForward, adj_sr, ricker
    z = load_golden("geometry")
    for i in range(3):
        f, dt, nt = z[f"ricker{i}_args"]
        np.testing.assert_array_equal(ricker(f, dt, int(nt)), z[f"ricker{i}"])
    base = dict(nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10)
    for i in range(8):
        n_grid, ns, ng, ss = z[f"sr{i}_args"]
        ctx = dict(base, n_grid=int(n_grid), ns=int(ns), ng=int(ng))
        fw = FWIForward(ctx, "cpu", sample_spatial=float(ss))
        c = fw.ctx
        isx, isz, igx, igz = adj_sr(c["sx"], c["sz"], c["gx"], c["gz"], c["dx"], c["nbc"])
        np.testing.assert_array_equal(isx, z[f"sr{i}_isx"])
        np.testing.assert_array_equal(igx, z[f"sr{i}_igx"])
        assert [isz, igz] == list(z[f"sr{i}_isz_igz"])
    ctx = dict(base, n_grid=16, nbc=8, ng=16, ns=3, sx=[0, 7.5, 15], gx=list(range(0, 16, 3)))
    fw = FWIForward(ctx, "cpu")
    c = fw.ctx
    isx, isz, igx, igz = adj_sr(c["sx"], c["sz"], c["gx"], c["gz"], c["dx"], c["nbc"])
    np.testing.assert_array_equal(isx, z["srx_isx"])
    np.testing.assert_array_equal(igx, z["srx_igx"])


def test_ricker_too_short_raises_like_reference():
    from red_diffeq.solvers.pde import ricker
    with pytest.raises(ValueError):
        ricker(15.0, 1e-3, 100)   # 147-sample wavelet does not fit


def test_oracle_geometry_matches_product():
    from oracle import oracle as O
    from red_diffeq.solvers.pde import ricker
    np.testing.assert_array_equal(O.ricker(15.0, 1e-3, 1000), ricker(15.0, 1e-3, 1000))


@pytest.mark.parametrize("name", ["loop_noise_small", "loop_laplace_small"])
def test_noise_and_missing_traces_vs_reference(name):
    """add_noise_to_seismic + missing_trace (utils/data_trans.py:33-62,110-153) with the reference's
    draws replayed: same draw order (noise, then one randperm per model), same arithmetic
    (Gaussian scale / Laplace inverse transform), the same receivers zeroed for every shot."""
    from conftest import replay_draws
    from red_diffeq.utils.data_trans import add_noise_to_seismic, missing_trace
    z = load_golden(name)
    std, missing = float(z["params"][5]), int(z["params"][4])
    with replay_draws(z):
        y = add_noise_to_seismic(torch.from_numpy(z["y"]), std, noise_type=str(z["noise_type"]))
        y, mask = missing_trace(y, missing, return_mask=True)
    assert np.array_equal(y.numpy(), z["y_noisy"])
    assert np.array_equal(mask.numpy(), z["mask"])
    m = z["mask"]
    assert (m == m[:, :1]).all() and (m == m[:, :, :1]).all()     # per receiver, not per shot/time
    assert ((m[:, 0, 0] == 0).sum(1) == missing).all()


def test_prepare_initial_model_vs_reference():
    from red_diffeq.utils.data_trans import prepare_initial_model
    z = load_golden("initial_models")
    for i in range(2):
        v = torch.from_numpy(z[f"v{i}"])
        assert np.array_equal(prepare_initial_model(v, "smoothed", sigma=10.0).numpy(), z[f"v{i}_smoothed"])
        assert np.array_equal(prepare_initial_model(v, "homogeneous").numpy(), z[f"v{i}_homogeneous"])
        assert np.array_equal(prepare_initial_model(v, "linear").numpy(), z[f"v{i}_linear"])
    with pytest.raises(AssertionError):
        prepare_initial_model(v, "constant")


def test_checkpoint_fixture_keys_and_weights_regenerate():
    """The dim-64 checkpoint fixture's 296 keys / shapes are this package's GaussianDiffusion
    state_dict, and tests/golden/ckpt_weights.py regenerates every weight deterministically."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from ckpt_weights import synth_param
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    z = load_golden("ckpt_dim64")
    d = GaussianDiffusion(Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1), image_size=72, timesteps=1000,
                          sampling_timesteps=250, objective="pred_noise")
    sd = d.state_dict()
    assert list(sd.keys()) == [str(k) for k in z["keys"]] and len(sd) == 296
    for k, shp in zip(z["keys"], z["shapes"]):
        assert tuple(sd[str(k)].shape) == tuple(int(s) for s in shp if s) or sd[str(k)].dim() == 0
    a = synth_param("model.init_conv.weight", (64, 1, 7, 7))
    assert np.array_equal(a, synth_param("model.init_conv.weight", (64, 1, 7, 7)))


def test_configs_load_unchanged():
    from red_diffeq.config import get_config, load_config, save_config
    cfg_dir = os.path.join(ROOT, "tests", "golden", "configs")
    c = get_config()
    assert c.pde.nbc == 120 and c.model.dim_mults == (1, 2, 4, 8)
    assert getattr(c.optimization, "fixed_timestep", 1) is None
    p = os.path.join(cfg_dir, "roundtrip.yaml")
    save_config(c, p)
    c2 = load_config(p)
    assert c2.pde.to_dict() == c.pde.to_dict() and list(c2.model.dim_mults) == [1, 2, 4, 8]
    os.remove(p)


def test_schedule_buffers_vs_reference():
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    z = load_golden("red_dim8")
    net = Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1)
    d = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250, objective="pred_noise")
    sd = d.state_dict()
    for k in z.files:
        if k.startswith("buf."):
            assert torch.equal(sd[k[4:]], torch.from_numpy(z[k])), k


def test_unet_state_dict_keys_match_reference():
    from red_diffeq.models.diffusion import Unet
    z = load_golden("unet_dim8")
    ref = {k[3:]: z[k].shape for k in z.files if k.startswith("sd.")}
    net = Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1)
    mine = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    assert mine == {k: tuple(v) for k, v in ref.items()}


def test_calculate_patches_vs_reference():
    from red_diffeq.regularization.diffusion import calculate_patches
    z = load_golden("small_losses")
    pos, ov = calculate_patches(190, 70)
    np.testing.assert_array_equal(np.array(pos), z["patches_190_70"])
    np.testing.assert_array_equal(np.array(ov), z["overlaps_190_70"])
    assert calculate_patches(70, 70) == ([(0, 70)], [])


def test_c_abi_library_exports_every_header_symbol():
    from red_diffeq import _hip
    lib = _hip.load_library()
    import glob
    hdr = "".join(open(h).read() for h in glob.glob(os.path.join(ROOT, "include", "*.h")))
    names = set(re.findall(r"^(?:int|size_t)\s+(rdq_\w+)\(", hdr, flags=re.M))
    assert names == set(_hip.SIGNATURES), names ^ set(_hip.SIGNATURES)
    for n in names:
        assert isinstance(getattr(lib, n), ctypes._CFuncPtr)
    # host-only entry points work without a GPU
    assert lib.rdq_l1_partial_bytes(2, 100000) == 2 * 25 * 2 * 8
    assert lib.rdq_fwi_plan_destroy(None) == 0


def test_c_abi_rejects_bad_geometry():
    from red_diffeq import _hip
    lib = _hip.load_library()
    isx = (ctypes.c_int32 * 1)(500)   # outside the padded grid
    igx = (ctypes.c_int32 * 1)(3)
    wav = (ctypes.c_double * 10)()
    g = _hip.FwiGeom(nz=4, nx=4, nbc=2, nt=10, ns=1, ng=1, sample_temporal=1, dx=10.0, dt=1e-3, isz=2, igz=2,
                     isx=isx, igx=igx, wavelet=wav)
    h = ctypes.c_void_p()
    assert lib.rdq_fwi_plan_create(ctypes.byref(g), ctypes.byref(h)) == -10001


def test_no_cpu_fallback():
    from red_diffeq.core.losses import l1_misfit
    from red_diffeq.regularization.benchmark import total_variation_loss
    from red_diffeq.solvers.pde import FWIForward
    ctx = dict(n_grid=8, nt=200, dx=10.0, dt=0.001, nbc=4, f=15.0, sz=10, gz=10, ng=8, ns=1)
    fwi = FWIForward(ctx, "cpu", normalize=False)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        fwi(torch.zeros(1, 1, 8, 8))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        total_variation_loss(torch.zeros(1, 1, 8, 8))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        l1_misfit(torch.zeros(1, 4), torch.zeros(1, 4))


def test_synthetic_models_in_range():
    from red_diffeq.utils.synthetic import make_model
    for fam in ("flatvel", "curvevel", "curvefault"):
        v = make_model(fam, 70, 70, seed=8888, batch=2)
        assert v.shape == (2, 1, 70, 70) and v.min() >= 1500 and v.max() <= 4500


def test_cosine_lr_matches_torch_scheduler():
    """Host-side CosineAnnealingLR restatement used by the fused loop (inversion.py:81)."""
    from red_diffeq.core.fused import CosineLR
    for T, steps in ((300, 310), (7, 40)):
        p = torch.zeros(1, requires_grad=True)
        opt = torch.optim.SGD([p], lr=0.03)
        sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=T, eta_min=0.0)
        mine = CosineLR(0.03, T_max=T)
        for _ in range(steps):
            opt.step()
            sch.step()
            assert mine.step() == opt.param_groups[0]["lr"]


def _reference_blend(gp, pos, ov, B, shape):
    """The reference's per-patch blending loop (regularization/diffusion.py:128-147), restated."""
    grad = torch.zeros(shape)
    wmap = torch.zeros(shape)
    for i, (a, b) in enumerate(pos):
        w = torch.ones(b - a)
        if i > 0:
            w[:ov[i - 1]] = 0.5
        if i < len(pos) - 1:
            w[-ov[i]:] = 0.5
        w = w.view(1, 1, 1, -1)
        grad[:, :, :, a:b] += gp[i * B:(i + 1) * B] * w
        wmap[:, :, :, a:b] += w
    return grad / wmap.clamp(min=1e-8)


@pytest.mark.parametrize("W", [190, 140, 71, 300])
def test_tile_plan_width_windows_bitexact_vs_reference_loop(W):
    """Height <= 70 (Marmousi 70x190): gather / blend by index == the reference's loop, bit for bit
    (W = 140 has an empty overlap, where the reference halves a whole window)."""
    from red_diffeq.regularization.diffusion import calculate_patches, tile_plan
    B, H = 2, 70
    g = torch.Generator().manual_seed(W)
    mu = torch.randn(B, 1, H, W, generator=g)
    tp = tile_plan(H, W, 70, B, "cpu")
    pos, ov = calculate_patches(W, H)
    ref_x = torch.cat([mu[:, :, :, a:b] for a, b in pos], dim=0)
    assert torch.equal(tp.gather(mu), ref_x)
    gp = torch.randn(ref_x.shape, generator=g)
    got = tp.assemble(gp)
    ref = _reference_blend(gp, pos, ov, B, mu.shape)
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("H,W", [(500, 3000), (140, 140), (100, 190), (71, 71)])
def test_tile_plan_2d_covers_and_round_trips(H, W):
    """2-D tiles (configs[4]): every pixel covered by 1..4 tiles of 70x70, and blending the tiles of a
    field gathers it back exactly (at a pixel every covering tile has the same weight)."""
    from red_diffeq.regularization.diffusion import tile_plan
    B = 1
    tp = tile_plan(H, W, 70, B, "cpu")
    assert (tp.mh, tp.mw) == (70, 70)
    x = torch.randn(B, 1, H, W, generator=torch.Generator().manual_seed(H * W))
    t = tp.gather(x)
    assert t.shape == (tp.P * B, 1, 70, 70)
    assert torch.equal(tp.assemble(t), x)
    if (H, W) == (500, 3000):
        assert tp.P == 8 * 43


def test_diffusion_bench_patch_split_merge_and_smoothing():
    """DiffusionFWI host helpers (reference diffusion_bench/diffusionfwi.py:32-76, 289-295):
    split -> merge round-trips with overlapping patches, the fold-based merge equals the reference's
    loop, and the device Gaussian smoothing equals scipy.ndimage.gaussian_filter (reflect)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
    from scipy.ndimage import gaussian_filter
    from diffusion_bench.diffusionfwi import _gaussian_smooth, merge_patches_to_data, split_data_to_patches
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 1, 20, 30, generator=g)
    k, st = [8, 10], [4, 5]
    p = split_data_to_patches(x, k, st)
    assert p.shape == (((20 - 8) // 4 + 1) * ((30 - 10) // 5 + 1), 1, 8, 10)
    torch.testing.assert_close(merge_patches_to_data(p, [20, 30], k, st), x, rtol=0, atol=1e-6)
    q = p * torch.rand(p.shape, generator=g)                  # reference loop (diffusionfwi.py:56-76)
    merged = torch.zeros(1, 1, 20, 30)
    count = torch.zeros(1, 1, 20, 30)
    idx = 0
    for i in range((20 - 8) // 4 + 1):
        for j in range((30 - 10) // 5 + 1):
            merged[:, :, i * 4:i * 4 + 8, j * 5:j * 5 + 10] += q[idx]
            count[:, :, i * 4:i * 4 + 8, j * 5:j * 5 + 10] += 1
            idx += 1
    torch.testing.assert_close(merge_patches_to_data(q, [20, 30], k, st), merged / count.clamp(min=1),
                               rtol=1e-6, atol=1e-6)
    gr = torch.randn(2, 1, 16, 21, generator=g)
    for s in (0.7, 1.0, 2.5):
        ref = gaussian_filter(gr.numpy().astype(np.float64), sigma=[0, 0, s, s])
        np.testing.assert_allclose(_gaussian_smooth(gr, s).numpy(), ref, rtol=1e-5, atol=1e-6)


def test_ilvr_resampler_vs_reference_fixture():
    """ILVR's bicubic antialiased resampler restated as per-axis weight matrices
    (diffusion_bench/ilvr_fwi.py) vs the reference's Resizer outputs (tests/golden/ilvr_small.npz,
    made by running diffusion_bench/resizer.py), down by 1/N and back up, N in {16, 9, 5, 2}."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
    from diffusion_bench.ilvr_fwi import resize
    z = load_golden("ilvr_small")
    x = torch.from_numpy(z["rz_x"])
    for n in (16, 9, 5, 2):
        d = resize(x, 1.0 / n)
        np.testing.assert_allclose(d.numpy(), z[f"rz_down{n}"], rtol=0, atol=1e-6)
        u = resize(torch.from_numpy(z[f"rz_down{n}"]), float(n), in_hw=(int(70 / n), int(70 / n)))
        np.testing.assert_allclose(u.numpy(), z[f"rz_up{n}"], rtol=0, atol=1e-6)


def test_bench_launches_n_ranks_itself(monkeypatch):
    """bench.py --gpus N outside a launcher starts N ranks via torch.distributed.run (child
    processes; the parent never initialises the GPU) and exits with their status."""
    import importlib.util
    import subprocess
    import sys
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    seen = {}
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: seen.update(cmd=cmd, env=env) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_fallback_restores_each_plans_own_persistent_mode():
    """re-promotion after a persistent fault puts back every plan's own mode.  A plan
    pinned to the chunked kernels stays chunked, a plan pinned to one region class keeps it, and the
    fault-path test mode (-1) comes back as auto (1).  Stub plans: only set_persistent / status_t are
    touched, so no GPU is needed."""
    from red_diffeq.solvers.pde import FWIForward, FwiPlan

    class Stub:
        def __init__(self, mode):
            self.persist_mode, self._saved_mode, self.status_t = mode, None, torch.ones(4)
            self.calls = []

        set_persistent = FwiPlan.set_persistent
        _set_mode = FwiPlan._set_mode

        @property
        def lib(self):
            stub = self

            class L:
                def rdq_fwi_set_persistent(self, h, mode):
                    stub.calls.append(mode)
                    return 0
            return L()

        handle = None

    ctx = dict(n_grid=70, ns=2, ng=70, dx=10.0, nt=200, nbc=20, f=15.0, dt=0.001, sz=10, gz=10)
    fwi = FWIForward(ctx, torch.device("cpu"))
    pinned, failing, cls12 = Stub(0), Stub(-1), Stub(12)
    fwi._plans = {"a": pinned, "b": failing, "c": cls12}
    fwi.fallback_to_chunked()
    fwi.fallback_to_chunked()                  # a second fault before the restore keeps the saved modes
    assert [p.persist_mode for p in (pinned, failing, cls12)] == [0, 0, 0]
    assert all(float(p.status_t.sum()) == 0 for p in (pinned, failing, cls12))
    fwi.restore_persistent()
    assert [p.persist_mode for p in (pinned, failing, cls12)] == [0, 1, 12]
    assert all(p._saved_mode is None for p in (pinned, failing, cls12))
    fwi.restore_persistent()                   # nothing saved: no change
    assert [p.persist_mode for p in (pinned, failing, cls12)] == [0, 1, 12]
    # a direct set_persistent during the fallback is the mode the restore brings back
    fwi.fallback_to_chunked()
    cls12.set_persistent(8)
    assert cls12.persist_mode == 8
    fwi.restore_persistent()
    assert [p.persist_mode for p in (pinned, failing, cls12)] == [0, 1, 8]


def test_plan_created_during_fallback_starts_chunked(monkeypatch):
    """a plan created while the operator is fallen back (a new grid shape) runs the chunked
    kernels until restore_persistent(), which gives it back its own (auto) mode.  FwiPlan is replaced by a
    stub, so no GPU is needed."""
    from red_diffeq.solvers import pde

    class Stub:
        def __init__(self, *a, **k):
            self.persist_mode, self._saved_mode, self.status_t = 1, None, torch.ones(4)

        set_persistent = pde.FwiPlan.set_persistent
        _set_mode = pde.FwiPlan._set_mode
        handle = None

        @property
        def lib(self):
            class L:
                def rdq_fwi_set_persistent(self, h, mode):
                    return 0
            return L()

    monkeypatch.setattr(pde, "FwiPlan", Stub)
    ctx = dict(n_grid=70, ns=2, ng=70, dx=10.0, nt=200, nbc=20, f=15.0, dt=0.001, sz=10, gz=10)
    fwi = pde.FWIForward(ctx, torch.device("cpu"))
    old = fwi._plan(70, 70, torch.device("cpu"))
    fwi.fallback_to_chunked()
    new = fwi._plan(70, 90, torch.device("cpu"))
    assert old.persist_mode == 0 and new.persist_mode == 0
    fwi.restore_persistent()
    assert old.persist_mode == 1 and new.persist_mode == 1
    again = fwi._plan(70, 110, torch.device("cpu"))
    assert again.persist_mode == 1


def test_unet_options_are_atomic_and_versioned():
    """rdq_unet_set_option returns the previous value, rejects unknown options and bad values,
    and every change bumps rdq_unet_options_generation (the U-Net's captured-graph cache key), while a
    set to the current value does not.  Host-only: no GPU call."""
    from red_diffeq import _hip
    lib = _hip.load_library()
    g0 = lib.rdq_unet_options_generation()
    old = lib.rdq_unet_set_option(6, 5)               # RDQ_UNET_OPT_CC_MIN_STAGES
    try:
        assert old == 3
        assert lib.rdq_unet_options_generation() == g0 + 1
        assert lib.rdq_unet_set_option(6, 5) == 5 and lib.rdq_unet_options_generation() == g0 + 1
        assert lib.rdq_unet_set_option(6, 0) < 0 and lib.rdq_unet_set_option(99, 1) < 0
    finally:
        assert lib.rdq_unet_set_option(6, old) == 5
    assert lib.rdq_unet_options_generation() == g0 + 2


def test_k12_covers_only_the_reference_ssim():
    """the engine evaluates SSIM with the fused K12 kernel only when the caller's
    ssim_loss is the reference's 11 x 11, sigma 1.5 SSIM module (either size_average); any other
    module -- another window, a subclass, a modified window -- is called as the reference's
    MetricsCalculator calls it (reference core/metrics.py:13-46)."""
    from red_diffeq.core.inversion import k12_covers
    from red_diffeq.utils.ssim import SSIM
    assert k12_covers(SSIM(window_size=11))
    assert k12_covers(SSIM(window_size=11, size_average=False))
    assert not k12_covers(SSIM(window_size=7))
    assert not k12_covers(None)

    class MySSIM(SSIM):
        pass
    assert not k12_covers(MySSIM(window_size=11))
    s = SSIM(window_size=11)
    s.window = s.window * 1.01
    assert not k12_covers(s)
