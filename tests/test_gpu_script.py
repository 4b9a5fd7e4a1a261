"""scripts/run_inversion.py (drop-in for the reference's scripts/run_inversion.py) end to end on a
tiny synthetic OpenFWI-layout dataset: config schema, mmap loader, batching, the
{idx}_results.npz writer (reference run_inversion.py:180-216), and equality with a direct
InversionEngine run under the same seed."""
import importlib.util
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _script():
    spec = importlib.util.spec_from_file_location("run_inversion", os.path.join(ROOT, "scripts", "run_inversion.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_run_inversion_script_tiny_dataset(cuda, tmp_path):
    from red_diffeq import get_config
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.synthetic import make_model
    ri = _script()
    cfg = get_config()
    cfg.pde.nt = 200
    cfg.pde.ns = 2
    cfg.model.dim = 8
    cfg.optimization.ts = 3
    cfg.optimization.regularization = "tv"
    cfg.optimization.reg_lambda = 0.01
    cfg.experiment.random_seed = 8888
    root = tmp_path / "dataset" / "OpenFWI"
    (root / "Seismic_Data").mkdir(parents=True)
    (root / "Velocity_Data").mkdir(parents=True)
    vel = make_model("flatvel", 70, 70, seed=3, batch=3)
    fwi = FWIForward(cfg.pde.to_dict(), cuda, normalize=True, v_denorm_func=v_denormalize,
                     s_norm_func=s_normalize_none)
    with torch.no_grad():
        seis = fwi(v_normalize(torch.from_numpy(vel)).to(cuda)).cpu().numpy()
    np.save(root / "Seismic_Data" / "FV.npy", seis)
    np.save(root / "Velocity_Data" / "FV.npy", vel)
    cfg.data.seismic_data_dir = str(root / "Seismic_Data")
    cfg.data.velocity_data_dir = str(root / "Velocity_Data")
    cfg.data.batch_size = 2
    cfg.experiment.results_dir = str(tmp_path / "out")
    cfg.experiment.name = "tiny"
    cfg.diffusion.model_path = str(tmp_path / "absent.pt")
    out = ri.run_experiment(cfg)
    files = sorted((out / "FV").glob("*_results.npz"))
    assert [f.name for f in files] == ["0_results.npz", "1_results.npz", "2_results.npz"]
    z = np.load(files[1])
    assert set(z.files) == {"result", "initial_velocity", "ground_truth", "total_losses", "obs_losses",
                            "reg_losses", "ssim", "mae", "rmse"}
    assert z["result"].shape == (70, 70) and z["ssim"].shape == (3,)
    np.testing.assert_array_equal(z["ground_truth"], vel[1, 0])
    assert (out / "config.yaml").exists()
    # the same batch through InversionEngine directly, same seed -> identical result
    from red_diffeq import InversionEngine, SSIM, prepare_initial_model, set_seed
    set_seed(cfg.experiment.random_seed, verbose=False)
    diff = ri.load_diffusion_model(cfg, cuda)
    eng = InversionEngine(diff, SSIM(), "tv", show_progress=False)
    v = torch.from_numpy(vel[0:2]).float()
    init = torch.cat([torch.nn.functional.pad(prepare_initial_model(v[i:i + 1], "smoothed", sigma=10.0),
                                              (1, 1, 1, 1)) for i in range(2)])
    mu, res = eng.optimize(init, v, torch.from_numpy(seis[0:2]).to(cuda), ri.initialize_forward_operator(cfg, cuda),
                           ts=3, lr=cfg.optimization.lr, reg_lambda=0.01, regularization="tv")
    np.testing.assert_array_equal(mu[1, 0].detach().cpu().numpy(), z["result"])
    np.testing.assert_array_equal(np.array(res[1]["rmse"]), z["rmse"])


@pytest.mark.parametrize("method", ["diffusionfwi", "ilvr"])
def test_run_bench_script_tiny_dataset(cuda, tmp_path, method):
    """scripts/run_bench.py (drop-in for diffusion_bench/run_bench.py): both methods over a tiny
    OpenFWI-layout dataset, the reference's results layout and keys (run_bench.py:152-183)."""
    import sys
    from red_diffeq import get_config
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.synthetic import make_model
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    spec = importlib.util.spec_from_file_location("run_bench", os.path.join(ROOT, "scripts", "run_bench.py"))
    rb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rb)
    cfg = get_config()
    cfg.pde.nt = 200
    cfg.pde.ns = 2
    cfg.model.dim = 8
    cfg.optimization.ts = 2
    cfg.optimization.diffusion_ts = 3
    cfg.experiment.random_seed = 8888
    root = tmp_path / "dataset" / "OpenFWI"
    (root / "Seismic_Data").mkdir(parents=True)
    (root / "Velocity_Data").mkdir(parents=True)
    vel = make_model("curvevel", 70, 70, seed=4, batch=2)
    fwi = FWIForward(cfg.pde.to_dict(), cuda, normalize=True, v_denorm_func=v_denormalize,
                     s_norm_func=s_normalize_none)
    with torch.no_grad():
        seis = fwi(v_normalize(torch.from_numpy(vel)).to(cuda)).cpu().numpy()
    np.save(root / "Seismic_Data" / "CV.npy", seis)
    np.save(root / "Velocity_Data" / "CV.npy", vel)
    cfg.data.seismic_data_dir = str(root / "Seismic_Data")
    cfg.data.velocity_data_dir = str(root / "Velocity_Data")
    cfg.data.batch_size = 2
    cfg.experiment.results_dir = str(tmp_path / "out")
    cfg.experiment.name = "bench_" + method
    cfg.diffusion.model_path = str(tmp_path / "absent.pt")
    out = rb.run_experiment(cfg, method=method)
    files = sorted((out / "CV").glob("*_results.npz"))
    assert [f.name for f in files] == ["0_results.npz", "1_results.npz"]
    z = np.load(files[0])
    assert set(z.files) == {"result", "initial_velocity", "ground_truth", "total_losses", "obs_losses", "ssim",
                            "mae", "rmse"}
    assert z["result"].shape == (70, 70) and z["rmse"].shape == (3,)
    assert np.isfinite(z["result"]).all() and np.abs(z["result"]).max() <= 1.0


def test_checkpoint_round_trip_dim64(cuda, tmp_path):
    """A dim-64 checkpoint in the reference's layout ({"model": GaussianDiffusion.state_dict(), ...},
    models/diffusion.py:617-625) read by the drop-in loader (reference run_inversion.py:63-67):
    all 296 keys load, the checkpoint's schedule buffers (a LINEAR beta schedule) override the
    sigmoid ones the constructor computes, and eps-hat / model_predictions match the reference's
    outputs for the same weights (tests/golden/ckpt_dim64.npz, tests/golden/ckpt_weights.py)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from ckpt_weights import synth_param
    from conftest import load_golden
    from red_diffeq import get_config
    z = load_golden("ckpt_dim64")
    sd = {}
    for k, shp in zip(z["keys"], z["shapes"]):
        k = str(k)
        sd[k] = (torch.from_numpy(z["buf." + k]) if "buf." + k in z.files
                 else torch.from_numpy(synth_param(k, [int(s) for s in shp if s])))
    path = tmp_path / "model-x.pt"
    torch.save({"step": 7, "model": sd, "version": "2.1.1"}, path)
    cfg = get_config()
    cfg.diffusion.model_path = str(path)
    diff = _script().load_diffusion_model(cfg, cuda)
    assert torch.equal(diff.alphas_cumprod.cpu(), torch.from_numpy(z["buf.alphas_cumprod"]))
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["t"]).to(cuda)
    with torch.no_grad():
        eps = diff.model(x, t, None)
        pred = diff.model_predictions(x, t, x_self_cond=None, clip_x_start=True, rederive_pred_noise=True)
    for got, key in ((eps, "eps"), (pred.pred_noise, "pred_noise"), (pred.pred_x_start, "pred_x_start")):
        ref = torch.from_numpy(z[key]).to(cuda)
        err = (got - ref).abs().max().item()
        assert err <= 2e-4 * ref.abs().max().item(), (key, err)


@pytest.mark.parametrize("name,n_models,nz,nx,family", [
    ("default", 2, 70, 70, "FV"),                # regularization none, batch_size 1 -> two batches
    ("openfwi_red-diffeq", 25, 70, 70, "CF"),    # RED-DiffEq, batch_size 25: 25 models x 5 shots, B = 25 U-Net
    ("marmousi_red-diffeq", 1, 70, 190, "Marmousi"),   # RED-DiffEq on 70 x 190: patched regulariser
])
def test_reference_configs_run_unchanged_through_cli(cuda, tmp_path, monkeypatch, name, n_models, nz, nx, family):
    """The reference's own configs (configs/default.yaml, configs/openfwi/red-diffeq.yaml,
    configs/marmousi/red-diffeq.yaml; parsed values in tests/golden/configs/*.json, written back out
    as YAML) through scripts/run_inversion.py's command line, main(["--config", ..., "--ts", "2"]),
    unchanged: their relative data / checkpoint / results paths resolve under a scratch directory
    holding a tiny synthetic dataset in the OpenFWI layout (the checkpoint is absent: random U-Net).
    Every model of every batch writes <idx>_results.npz with the reference's keys
    (reference run_inversion.py:180-216, 332-415), and each file equals, bit for bit, a direct
    InversionEngine.optimize call on the same inputs under the same seed (the CLI adds no
    numerics of its own; the B = 25 numbers themselves are pinned against the reference engine by
    test_gpu_loop_parity.py::test_red_loop_openfwi_yaml_b25)."""
    import json
    import yaml
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.synthetic import make_model
    cfg = json.load(open(os.path.join(ROOT, "tests", "golden", "configs", name + ".json")))["config"]
    monkeypatch.chdir(tmp_path)
    with open("config.yaml", "w") as f:
        yaml.safe_dump(cfg, f)
    seis_dir, vel_dir = cfg["data"]["seismic_data_dir"], cfg["data"]["velocity_data_dir"]
    os.makedirs(seis_dir)
    os.makedirs(vel_dir)
    vel = make_model({"FV": "flatvel", "CF": "curvefault"}.get(family, "curvefault"), nz, nx, seed=5, batch=n_models)
    fwi = FWIForward(dict(cfg["pde"]), cuda, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    with torch.no_grad():
        seis = fwi(v_normalize(torch.from_numpy(vel)).to(cuda)).cpu().numpy()
    assert seis.shape == (n_models, cfg["pde"]["ns"], cfg["pde"]["nt"], cfg["pde"]["ng"])
    np.save(os.path.join(seis_dir, family + ".npy"), seis)
    np.save(os.path.join(vel_dir, family + ".npy"), vel)
    del fwi
    _script().main(["--config", "config.yaml", "--ts", "2"])
    runs = sorted((tmp_path / cfg["experiment"]["results_dir"]).glob(f"*/{cfg['experiment']['name']}/*"))
    assert len(runs) == 1, runs
    assert (runs[0] / "config.yaml").exists()
    files = sorted((runs[0] / family).glob("*_results.npz"), key=lambda p: int(p.name.split("_")[0]))
    assert [f.name for f in files] == [f"{i}_results.npz" for i in range(n_models)]
    for f in (files[0], files[-1]):
        z = np.load(f)
        assert set(z.files) == {"result", "initial_velocity", "ground_truth", "total_losses", "obs_losses",
                                "reg_losses", "ssim", "mae", "rmse"}
        assert z["result"].shape == (nz, nx) and z["obs_losses"].shape == (2,)
        idx = int(f.name.split("_")[0])
        np.testing.assert_array_equal(z["ground_truth"], vel[idx, 0])
    # the same run as direct engine calls: seed, random-initialised U-Net, operator, engine, then every
    # batch in file order (the engine's draws continue across batches as in the script)
    from red_diffeq import GaussianDiffusion, InversionEngine, SSIM, Unet, prepare_initial_model
    from red_diffeq.utils.seed_utils import set_seed
    c = cfg
    set_seed(c["experiment"]["random_seed"], verbose=False)
    m = c["model"]
    diff = GaussianDiffusion(Unet(dim=m["dim"], dim_mults=tuple(m["dim_mults"]), flash_attn=m["flash_attn"],
                                  channels=m["channels"]),
                             image_size=c["diffusion"]["image_size"], timesteps=c["diffusion"]["timesteps"],
                             sampling_timesteps=c["diffusion"]["sampling_timesteps"],
                             objective=c["diffusion"]["objective"]).to(cuda).eval()
    fwi = FWIForward(dict(cfg["pde"]), cuda, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    o = c["optimization"]
    reg = o["regularization"] if o["regularization"] and o["regularization"] != "none" else None
    eng = InversionEngine(diff, SSIM(window_size=11, size_average=True), o["regularization"] or None,
                          use_time_weight=o.get("use_time_weight", False), sigma_x0=o.get("sigma_x0", 1e-4),
                          fixed_timestep=o.get("fixed_timestep"), show_progress=False)
    bsz = c["data"]["batch_size"]
    for s0 in range(0, n_models, bsz):
        s1 = min(s0 + bsz, n_models)
        v_b = torch.from_numpy(vel[s0:s1]).float()
        init = torch.cat([torch.nn.functional.pad(prepare_initial_model(v_b[i:i + 1], o["initial_type"], sigma=o["sigma"]),
                                                  (1, 1, 1, 1), "constant", 0) for i in range(s1 - s0)])
        mu, res = eng.optimize(init, v_b, torch.from_numpy(seis[s0:s1]).float().to(cuda), fwi, ts=2, lr=o["lr"],
                               reg_lambda=o["reg_lambda"], noise_std=o["noise_std"], noise_type=o["noise_type"],
                               missing_number=o["missing_number"], regularization=reg)
        mu = mu.detach().cpu().numpy()
        for i in range(s1 - s0):
            z = np.load(files[s0 + i])
            # (assert_array_equal treats NaN == NaN: the model's range is checked on its own)
            assert np.isfinite(z["result"]).all() and np.abs(z["result"]).max() <= 1.0
            for k in ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse"):
                assert np.isfinite(z[k]).all(), k
            np.testing.assert_array_equal(z["result"], mu[i, 0])
            np.testing.assert_array_equal(z["initial_velocity"], init[i, 0, 1:-1, 1:-1].numpy())
            for k in ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse"):
                np.testing.assert_array_equal(z[k], np.array(res[i][k]), err_msg=k)
