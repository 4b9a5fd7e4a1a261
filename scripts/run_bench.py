"""Drop-in for the reference's diffusion_bench/run_bench.py (SimingShan/red-diffeq): run the
DiffusionFWI or ILVR-FWI baseline over OpenFWI-layout data on the MI355X package.

Same command line (--method diffusionfwi|ilvr|ilvr_fwi, --config, --lr, --ts, --diffusion_ts,
--grad_norm, --grad_smooth, --model_blur, --grad_clip, --use_ilvr, --ilvr_weight,
--ilvr_down_schedule, --use_patches, --patch_height/--patch_width, --patch_stride_h/--patch_stride_w,
--noise_type, --noise_std, --sigma, --missing_number, --batch_size, --experiment_name,
--random_seed), same config keys (optimization.diffusion_ts and the gradient-trick keys with the
reference's defaults, run_bench.py:119-141) and the same output layout
(<results_dir>/<dataset>/<experiment>/<timestamp>/{config.yaml, <family>/<idx>_results.npz} with
result, initial_velocity, ground_truth, total_losses, obs_losses, ssim, mae, rmse; run_bench.py:152-183).
Data loading, model / operator construction and the config machinery are shared with
scripts/run_inversion.py."""
import argparse
import sys
from datetime import datetime
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "red-diffeq_amd"))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from tqdm import tqdm  # noqa: E402

import run_inversion as ri  # noqa: E402
from diffusion_bench import ILVR_FWI, DiffusionFWI  # noqa: E402
from red_diffeq import SSIM, get_config, load_config, prepare_initial_model, save_config  # noqa: E402


def _opt(cfg, key, default):
    return cfg.get(key, default) if hasattr(cfg, "get") else getattr(cfg, key, default)


def process_batch(s, e, seis_mmap, vel_mmap, config, bench, fwi_forward, device):
    seis = torch.from_numpy(np.array(seis_mmap[s:e])).float().to(device)
    vel = torch.from_numpy(np.array(vel_mmap[s:e])).float()
    init = torch.cat([prepare_initial_model(vel[i:i + 1], config.optimization.initial_type,
                                            sigma=config.optimization.sigma) for i in range(vel.shape[0])], dim=0)
    o = config.optimization
    kw = dict(ts=o.ts, diffusion_ts=o.diffusion_ts, lr=o.lr, noise_std=o.noise_std, noise_type=o.noise_type,
              missing_number=o.missing_number, grad_norm=_opt(o, "grad_norm", True),
              grad_smooth=_opt(o, "grad_smooth", None), model_blur=_opt(o, "model_blur", False),
              grad_clip=_opt(o, "grad_clip", 1.0), use_patches=_opt(o, "use_patches", False),
              patch_kernel_size=_opt(o, "patch_kernel_size", None), patch_stride=_opt(o, "patch_stride", None))
    if isinstance(bench, ILVR_FWI):
        kw.update(use_ilvr=_opt(o, "use_ilvr", True), ilvr_weight=_opt(o, "ilvr_weight", 0.05),
                  ilvr_down_schedule=_opt(o, "ilvr_down_schedule", "linear"))
    mu, results = bench.optimize(init, vel, seis, fwi_forward, **kw)
    return mu, results, init, vel


def save_batch_results(s, e, mu, results, init, vel, out_dir: Path):
    out_dir.mkdir(parents=True, exist_ok=True)
    mu_np, init_np, vel_np = mu.detach().cpu().numpy(), init.detach().cpu().numpy(), vel.cpu().numpy()
    for i, idx in enumerate(range(s, e)):
        m = results[i]
        np.savez(str(out_dir / f"{idx}_results.npz"), result=mu_np[i, 0], initial_velocity=init_np[i, 0],
                 ground_truth=vel_np[i, 0], **{k: np.array(m[k]) for k in ("total_losses", "obs_losses", "ssim",
                                                                              "mae", "rmse")})


def run_experiment(config, method="diffusionfwi") -> Path:
    seed = config.experiment.random_seed
    if seed is not None:
        from red_diffeq.utils.seed_utils import set_seed
        set_seed(seed, verbose=True)
    device = ri.setup_device()
    diffusion = ri.load_diffusion_model(config, device)
    fwi_forward = ri.initialize_forward_operator(config, device)
    ssim = SSIM(window_size=11, size_average=True)
    cls = ILVR_FWI if method.lower() in ("ilvr", "ilvr_fwi") else DiffusionFWI
    bench = cls(diffusion, fwi_forward, ssim)
    seismic_dir = Path(config.data.seismic_data_dir).resolve()
    dataset = seismic_dir.parts[-2] if len(seismic_dir.parts) >= 2 else None
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    base = Path(config.experiment.results_dir)
    results_dir = (base / dataset if dataset else base) / config.experiment.name / stamp
    results_dir.mkdir(parents=True, exist_ok=True)
    save_config(config, results_dir / "config.yaml")
    print(f"Results will be saved to: {results_dir}")
    for family in ri.get_data_files(config):
        seis_mmap = np.load(Path(config.data.seismic_data_dir) / family, mmap_mode="r")
        vel_mmap = np.load(Path(config.data.velocity_data_dir) / family, mmap_mode="r")
        n, bsz = seis_mmap.shape[0], config.data.batch_size
        for s in tqdm(range(0, n, bsz), desc=f"Batches ({family})"):
            e = min(s + bsz, n)
            mu, res, init, vel = process_batch(s, e, seis_mmap, vel_mmap, config, bench, fwi_forward, device)
            save_batch_results(s, e, mu, res, init, vel, results_dir / Path(family).stem)
    print(f"Experiment complete! Results saved to: {results_dir}")
    return results_dir


def main(argv=None):
    tf = lambda x: x.lower() == "true"  # noqa: E731
    p = argparse.ArgumentParser(description="Benchmark diffusion FWI methods (DiffusionFWI or ILVR-FWI)")
    p.add_argument("--method", choices=["diffusionfwi", "ilvr", "ilvr_fwi"], default="diffusionfwi")
    p.add_argument("--config", type=Path, default=None)
    for name, typ in (("lr", float), ("ts", int), ("diffusion_ts", int), ("grad_norm", tf), ("grad_smooth", float),
                      ("model_blur", tf), ("grad_clip", float), ("use_ilvr", tf), ("ilvr_weight", float),
                      ("ilvr_down_schedule", str), ("use_patches", tf), ("patch_height", int), ("patch_width", int),
                      ("patch_stride_h", int), ("patch_stride_w", int), ("noise_std", float), ("sigma", float),
                      ("missing_number", int), ("batch_size", int), ("experiment_name", str), ("random_seed", int)):
        p.add_argument("--" + name, type=typ)
    p.add_argument("--noise_type", choices=["gaussian", "laplace"])
    a = p.parse_args(argv)
    config = load_config(a.config) if a.config else get_config()
    o = config.optimization
    for k in ("lr", "ts", "diffusion_ts", "grad_norm", "grad_smooth", "model_blur", "grad_clip", "use_ilvr",
              "ilvr_weight", "ilvr_down_schedule", "use_patches", "noise_type", "noise_std", "sigma",
              "missing_number"):
        if getattr(a, k) is not None:
            o[k] = getattr(a, k)
    if a.patch_height is not None and a.patch_width is not None:
        o["patch_kernel_size"] = [a.patch_height, a.patch_width]
    if a.patch_stride_h is not None and a.patch_stride_w is not None:
        o["patch_stride"] = [a.patch_stride_h, a.patch_stride_w]
    if a.batch_size is not None:
        config.data.batch_size = a.batch_size
    if a.experiment_name is not None:
        config.experiment.name = a.experiment_name
    if a.random_seed is not None:
        config.experiment.random_seed = a.random_seed
    if "diffusion_ts" not in o:
        raise ValueError("optimization.diffusion_ts is required (config or --diffusion_ts)")
    return run_experiment(config, method=a.method)


if __name__ == "__main__":
    main()
