"""Drop-in for the reference's scripts/run_inversion.py (SimingShan/red-diffeq), running on the
MI355X package in red-diffeq_amd/.

Same command line (--config, --lr, --ts, --regularization, --reg_lambda, --noise_type, --noise_std,
--sigma, --sigma_x0, --missing_number, --batch_size, --experiment_name, --results_dir,
--random_seed, --openfwi_families, --sample_index), same config schema (the reference's
configs/*.yaml load unchanged), same data layout (OpenFWI family files <seismic_dir>/<F>.npy
(N, ns, nt, ng) and <velocity_dir>/<F>.npy (N, 1, nz, nx), memory-mapped) and the same output:
<results_dir>/<dataset>/<experiment>/<timestamp>/{config.yaml, <family>/<idx>_results.npz}
with keys result, initial_velocity, ground_truth, total_losses, obs_losses, reg_losses, ssim,
mae, rmse (reference run_inversion.py:180-216).

Differences by design: checkpoints are read with torch.load(weights_only=True); no
`accelerate` wrapper (it only wraps GaussianDiffusion.forward, the training loss, which the
inversion never calls); under torchrun (WORLD_SIZE > 1) the shots are sharded over the ranks
(one RCCL all-reduce of the data-term gradient per iteration) and rank 0 writes the
results.
"""
import argparse
import os
import sys
from datetime import datetime
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "red-diffeq_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from tqdm import tqdm  # noqa: E402

from red_diffeq import (FWIForward, GaussianDiffusion, InversionEngine, SSIM, Unet, get_config,  # noqa: E402
                        load_config, prepare_initial_model, s_normalize_none, save_config, v_denormalize)
from red_diffeq.config.config_dict import ConfigDict  # noqa: E402


def _dist():
    """(rank, world, local_rank); initialises the RCCL process group under torchrun."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if world > 1:
        return dist.get_rank(), world, int(os.environ.get("LOCAL_RANK", "0"))
    return 0, 1, 0


def setup_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("red-diffeq_amd runs on the MI355X (no ROCm device visible); there is no CPU path")
    _, _, local = _dist()
    device = torch.device("cuda", local)
    print(f"Using device: {device} ({torch.cuda.get_device_name(device)})")
    return device


def load_diffusion_model(config, device: torch.device) -> GaussianDiffusion:
    model = Unet(dim=config.model.dim, dim_mults=tuple(config.model.dim_mults),
                 flash_attn=config.model.flash_attn, channels=config.model.channels)
    diffusion = GaussianDiffusion(model, image_size=config.diffusion.image_size,
                                  timesteps=config.diffusion.timesteps,
                                  sampling_timesteps=config.diffusion.sampling_timesteps,
                                  objective=config.diffusion.objective).to(device)
    path = Path(config.diffusion.model_path)
    if path.exists():
        ckpt = torch.load(path, map_location=device, weights_only=True)
        diffusion.load_state_dict(ckpt["model"] if "model" in ckpt else ckpt)
        print(f"Loaded pretrained model from: {path}")
    else:
        print(f"WARNING: pretrained model not found at {path}; continuing with random initialisation")
    return diffusion.eval()


def initialize_forward_operator(config, device: torch.device) -> FWIForward:
    ctx = config.pde.to_dict()
    rank, world, _ = _dist()
    shots = None
    if world > 1:   # shot-parallel: rank r models shots [r*ns/N, (r+1)*ns/N)
        ns = int(ctx["ns"]) if "sx" not in ctx else len(ctx["sx"])
        shots = (rank * ns // world, (rank + 1) * ns // world)
    return FWIForward(ctx, device, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none,
                      shots=shots)


def get_data_files(config) -> list:
    seismic_dir = Path(config.data.seismic_data_dir)
    if not seismic_dir.exists():
        raise FileNotFoundError(f"Seismic data directory not found: {seismic_dir}")
    names = [f.name for f in sorted(seismic_dir.glob(config.data.data_pattern))]
    if not names:
        raise ValueError(f"No data files found matching {config.data.data_pattern} in {seismic_dir}")
    wanted = getattr(config.data, "openfwi_families", None)
    if not wanted:
        return names
    if isinstance(wanted, str):
        wanted = [wanted]
    wanted = [w if w.endswith(".npy") else f"{w}.npy" for w in wanted if w is not None]
    if not wanted:
        return names
    picked = [n for n in names if n in wanted]
    if not picked:
        raise ValueError(f"No matching families found. Requested: {wanted}, Available: {names}")
    return picked


def process_batch(batch_start, batch_end, seis_mmap, vel_mmap, config, inversion_engine, fwi_forward, device):
    seis = torch.from_numpy(np.array(seis_mmap[batch_start:batch_end])).float().to(device)
    vel = torch.from_numpy(np.array(vel_mmap[batch_start:batch_end])).float()
    init = torch.cat([torch.nn.functional.pad(
        prepare_initial_model(vel[i:i + 1], config.optimization.initial_type, sigma=config.optimization.sigma),
        (1, 1, 1, 1), "constant", 0) for i in range(vel.shape[0])], dim=0)   # 70x70 -> 72x72
    reg = config.optimization.regularization
    mu, results = inversion_engine.optimize(
        init, vel, seis, fwi_forward, ts=config.optimization.ts, lr=config.optimization.lr,
        reg_lambda=config.optimization.reg_lambda, noise_std=config.optimization.noise_std,
        noise_type=config.optimization.noise_type, missing_number=config.optimization.missing_number,
        regularization=reg if reg and reg != "none" else None)
    return mu, results, init, vel


def save_batch_results(batch_start, batch_end, mu_batch, results_per_model, initial_model_batch, vel_batch,
                       output_dir: Path) -> None:
    mu_np = mu_batch.detach().cpu().numpy()
    vel_np = vel_batch.cpu().numpy()
    init_np = initial_model_batch[:, :, 1:-1, 1:-1].detach().cpu().numpy()
    output_dir.mkdir(parents=True, exist_ok=True)
    for i, idx in enumerate(range(batch_start, batch_end)):
        m = results_per_model[i]
        np.savez(str((output_dir / f"{idx}_results.npz").resolve()),
                 result=mu_np[i, 0], initial_velocity=init_np[i, 0], ground_truth=vel_np[i, 0],
                 **{k: np.array(m[k]) for k in ("total_losses", "obs_losses", "reg_losses", "ssim", "mae", "rmse")})


def run_experiment(config) -> Path:
    rank, world, _ = _dist()
    seed = config.experiment.random_seed
    if seed is not None:
        from red_diffeq.utils.seed_utils import set_seed
        set_seed(seed, verbose=rank == 0)
    device = setup_device()
    diffusion = load_diffusion_model(config, device)
    fwi_forward = initialize_forward_operator(config, device)
    engine = InversionEngine(diffusion, SSIM(window_size=11, size_average=True),
                             config.optimization.regularization if config.optimization.regularization else None,
                             use_time_weight=getattr(config.optimization, "use_time_weight", False),
                             sigma_x0=getattr(config.optimization, "sigma_x0", 0.0001),
                             fixed_timestep=getattr(config.optimization, "fixed_timestep", None),
                             show_progress=rank == 0)
    seismic_dir = Path(config.data.seismic_data_dir).resolve()
    dataset = seismic_dir.parts[-2] if len(seismic_dir.parts) >= 2 else None
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    base = Path(config.experiment.results_dir)
    results_dir = (base / dataset if dataset else base) / config.experiment.name / stamp
    if rank == 0:
        results_dir.mkdir(parents=True, exist_ok=True)
        save_config(config, results_dir / "config.yaml")
        print(f"Results will be saved to: {results_dir}")
    for family in get_data_files(config):
        seis_mmap = np.load(Path(config.data.seismic_data_dir) / family, mmap_mode="r")
        vel_mmap = np.load(Path(config.data.velocity_data_dir) / family, mmap_mode="r")
        n = seis_mmap.shape[0]
        idx = getattr(config.data, "sample_index", None)
        if idx is not None:
            if idx < 0 or idx >= n:
                print(f"Warning: sample_index {idx} is out of range [0, {n - 1}]. Skipping {family}.")
                continue
            ranges = [(idx, idx + 1)]
        else:
            bsz = config.data.batch_size
            ranges = [(s, min(s + bsz, n)) for s in range(0, n, bsz)]
        fam_dir = results_dir / Path(family).stem
        for s, e in tqdm(ranges, desc=f"Batches ({family})", disable=rank != 0):
            mu, results, init, vel = process_batch(s, e, seis_mmap, vel_mmap, config, engine, fwi_forward, device)
            if rank == 0:
                save_batch_results(s, e, mu, results, init, vel, fam_dir)
    if rank == 0:
        print(f"Experiment complete! Results saved to: {results_dir}")
    return results_dir


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description="Run Full Waveform Inversion with RED-DiffEq (MI355X)",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--config", type=Path, default=None, help="Path to YAML configuration file")
    p.add_argument("--lr", type=float)
    p.add_argument("--ts", type=int)
    p.add_argument("--regularization", choices=["diffusion", "tv", "l2", "none"])
    p.add_argument("--reg_lambda", type=float)
    p.add_argument("--noise_type", choices=["gaussian", "laplace"])
    p.add_argument("--noise_std", type=float)
    p.add_argument("--sigma", type=float)
    p.add_argument("--sigma_x0", type=float)
    p.add_argument("--missing_number", type=int)
    p.add_argument("--batch_size", type=int)
    p.add_argument("--experiment_name", type=str)
    p.add_argument("--results_dir", type=Path)
    p.add_argument("--random_seed", type=int)
    p.add_argument("--openfwi_families", type=str, nargs="+")
    p.add_argument("--sample_index", type=int, default=None)
    a = p.parse_args(argv)
    config = load_config(a.config) if a.config else get_config()
    overrides = {"lr": ("optimization", "lr"), "ts": ("optimization", "ts"),
                 "regularization": ("optimization", "regularization"),
                 "reg_lambda": ("optimization", "reg_lambda"), "noise_type": ("optimization", "noise_type"),
                 "noise_std": ("optimization", "noise_std"), "sigma": ("optimization", "sigma"),
                 "sigma_x0": ("optimization", "sigma_x0"), "missing_number": ("optimization", "missing_number"),
                 "batch_size": ("data", "batch_size"), "experiment_name": ("experiment", "name"),
                 "results_dir": ("experiment", "results_dir"), "random_seed": ("experiment", "random_seed"),
                 "openfwi_families": ("data", "openfwi_families"), "sample_index": ("data", "sample_index")}
    for arg, (sec, key) in overrides.items():
        v = getattr(a, arg)
        if v is not None:
            setattr(getattr(config, sec), key, str(v) if isinstance(v, Path) else v)
    run_experiment(config)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    assert isinstance(get_config(), ConfigDict)
    main()
