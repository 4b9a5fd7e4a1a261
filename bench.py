#!/usr/bin/env python
"""Benchmark: OpenFWI 70x70 FWI gradient step on MI355X (BASELINE.json metric, configs[1]).

One step = one iteration of the InversionEngine loop body for config 2 (FlatVel-A, 8 shots per
GPU, nt = 1000, TV regulariser): HIP coefficient fields -> 1000 forward steps (store-all
history) -> L1 misfit -> TV -> hand-written adjoint (1000 steps) -> gradient finalize ->
[N>1: one RCCL all-reduce of the 20 KB model gradient] -> Adam -> clamp -> cosine LR.
Inputs (velocity model, observed data) are synthetic and resident in HBM before timing.

value = shot-timesteps/s over the whole job = N * ns_per_gpu * nt * B / (step time, max over
ranks).  Weak scaling.  N = 1: configs[1] (FlatVel-A, 8 shots).  N > 1: configs[3]'s shape
(CurveFault-B, 32 shots per GPU: 256 over 8 GPUs); the N = 1 line also reports that per-rank
workload on one GPU ("configs3_rank_workload") as the base of the scaling curve.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--ns S] [--family F] [--no-cpu-baseline]

--gpus N > 1 outside a torch.distributed launcher starts the N ranks itself (torch.distributed.run,
one process per GPU, RCCL) as child processes; this parent never touches the GPU.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
sys.path.insert(0, ROOT)

METRIC = "shot-timesteps/sec (fwd+adj) + per-iter FWI wallclock, OpenFWI 70×70"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFS = 157.3     # MI355X fp32 matrix peak, v_mfma_f32_*_f32 (MI355X_MICROARCH.md)
UNET_GFLOP_72 = 18.17          # conv GFLOP of one 72x72 dim-64 U-Net forward


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--ns", type=int, default=None,
                   help="shots per GPU (default: 8 at N=1, configs[1]; 32 at N>1, configs[3]: 256 shots over 8 GPUs)")
    p.add_argument("--family", default=None, help="synthetic model family (default flatvel at N=1, curvefault at N>1)")
    p.add_argument("--nt", type=int, default=1000)
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-loop", action="store_true", help="skip the InversionEngine per-iteration wallclock")
    p.add_argument("--cpu-sample-shots", type=int, default=4)
    p.add_argument("--cpu-sample-reps", type=int, default=12,
                   help="repetitions of the CPU sample gradient (~10 s of host work at the defaults)")
    p.add_argument("--no-red", action="store_true", help="skip the configs[2] RED-DiffEq loop timing")
    p.add_argument("--no-configs4", action="store_true", help="skip the configs[4] per-rank RED iteration")
    return p.parse_args()


def cpu_baseline(ctx, vtrue, nshots, reps):
    """Oracle (CPU restatement, OpenMP) forward+adjoint on a bounded sample of the workload:
    `reps` gradients of `nshots` shots each (host history of one gradient only)."""
    from oracle import oracle as O
    c = dict(ctx, ns=nshots)
    f = O.OracleFWI(c, 1)
    vn = ((vtrue - 1500) / 3000 * 2 - 1).astype(np.float32)
    y, _ = f.forward(vn)
    v0 = (vn * 0.9).astype(np.float32)
    t0 = time.perf_counter()
    for _ in range(reps):
        seis, cf = f.forward(v0, keep_history=True)
        _, ds = O.l1_loss(seis, y)
        f.finalize(cf, *f.adjoint(cf, ds))
        del cf
    dt = time.perf_counter() - t0
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": round(reps * nshots * c["nt"] / dt, 1), "unit": "shot-timesteps/s", "cores": cores,
            "kind": "port",
            "sample": f"oracle/fwi_oracle.c fwd+adj+finalize, {reps} gradients x {nshots} shots x {c['nt']} "
                      f"steps, 70x70 "
                      f"(310x310 padded), {dt:.2f} s"}


def loop_wallclock(fwi, mu0, vt, y, a, dev, world):
    """ms per iteration of InversionEngine.optimize (TV, lambda 0.01, lr 0.03), iterations
    warmup..warmup+steps, timed around the whole call minus a warmup-only call."""
    import types
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.utils.ssim import SSIM
    eng = InversionEngine(types.SimpleNamespace(device=dev), SSIM(), regularization="tv", show_progress=False)
    mu = torch.nn.functional.pad(mu0, (1, 1, 1, 1))
    y_all = y
    if world > 1:   # the engine shards by fwi.shots against the full observed array
        parts = [torch.empty_like(y) for _ in range(world)]
        dist.all_gather(parts, y.contiguous())
        y_all = torch.cat(parts, dim=1)

    def run(ts):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.optimize(mu, vt, y_all, fwi, ts=ts, lr=0.03, reg_lambda=0.01, regularization="tv")
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(max(a.warmup, 1))
    t_w = run(a.warmup)
    t_all = run(a.warmup + a.steps)
    return round((t_all - t_w) / a.steps * 1e3, 4)


def red_loop_wallclock(dev, a, ns=32, family="curvevel", batch=1):
    """configs[2]: CurveVel-A, 32 shots, the full RED-DiffEq loop (HIP forward + adjoint + U-Net
    regulariser + Adam + metrics) through the drop-in InversionEngine, lambda 0.75, lr 0.03,
    random-init U-Net (dim 64, mults 1,2,4,8: the reference architecture; no checkpoint offline).
    `batch` models are inverted together (configs/openfwi/red-diffeq.yaml: batch_size 25).
    Returns ms per iteration over iterations [warmup, warmup + steps)."""
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.ssim import SSIM
    from red_diffeq.utils.synthetic import make_model
    torch.manual_seed(8888)
    ctx = dict(n_grid=70, nt=a.nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=ns)
    fwi = FWIForward(dict(ctx), dev, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    vt = torch.from_numpy(make_model(family, 70, 70, seed=8888, batch=batch))
    with torch.no_grad():
        y = fwi(v_normalize(vt).to(dev))
    mu = torch.nn.functional.pad(torch.cat([prepare_initial_model(vt[i:i + 1], "smoothed", sigma=10.0)
                                            for i in range(batch)]), (1, 1, 1, 1))
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
    diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                             objective="pred_noise").to(dev)
    eng = InversionEngine(diff, SSIM(), regularization="diffusion", sigma_x0=1e-4, show_progress=False)

    def run(ts):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.optimize(mu, vt, y, fwi, ts=ts, lr=0.03, reg_lambda=0.75, regularization="diffusion")
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(1)
    t_w = run(a.warmup)
    t_all = run(a.warmup + a.steps)
    return round((t_all - t_w) / a.steps * 1e3, 3)


def rank_workload_rate(dev, a, nsl, family):
    """One rank's share of configs[3] (CurveFault-B, 32 of the 256 shots) on this GPU: the same
    gradient step as the N > 1 bench minus its all-reduce, shot-timesteps/s over `a.steps` steps.
    The N-GPU scaling efficiency on configs[3]'s shape is value(N) / (N x this)."""
    from red_diffeq.core.fused import CosineLR, FusedAdamClamp
    from red_diffeq.core.losses import l1_misfit
    from red_diffeq.regularization.benchmark import total_variation_loss
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.synthetic import make_model
    nt = a.nt
    ctx = dict(n_grid=70, nt=nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=nsl * 8)
    fwi = FWIForward(dict(ctx), dev, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none,
                     shots=(0, nsl))
    vt = torch.from_numpy(make_model(family, 70, 70, seed=8888, batch=1))
    with torch.no_grad():
        y = fwi(v_normalize(vt).to(dev))
    mu = torch.nn.functional.pad(prepare_initial_model(vt, "smoothed", sigma=10.0), (1, 1, 1, 1)).to(dev)
    mu.requires_grad_(True)
    opt = FusedAdamClamp(mu, lr=0.03, clamp=(-1.0, 1.0))
    sched = CosineLR(0.03, T_max=300, eta_min=0.0)
    nobs = torch.full((1,), float(nsl * 8 * nt * 70), device=dev)

    def step():
        loss = l1_misfit(fwi(mu[:, :, 1:-1, 1:-1]), y, None, nobs) + 0.01 * total_variation_loss(mu)
        opt.zero_grad()
        loss.sum().backward()
        opt.step()
        opt.lr = sched.step()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    fwi.check()
    return {"workload": f"configs[3] per-rank share: CurveFault-B, {nsl} of {nsl * 8} shots, nt={nt}, one GPU, "
                        "no all-reduce", "ms_per_step": round(dt * 1e3, 4),
            "shot_timesteps_per_s": round(nsl * nt / dt, 1), "kernels": fwi._plan(70, 70, dev).launch_info(1)}


def configs4_rank_workload(dev, a, nsl=16, ns_total=128, nz=500, nx=3000, iters=3):
    """One rank's share of configs[4] on this GPU: a Marmousi-size 500 x 3000 model (740 x 3240 padded),
    16 of the 128 shots (the 8-way sharding's per-GPU share), nt = 1000, one RED-DiffEq iteration of the
    drop-in InversionEngine (HIP forward + adjoint on the chunked wide-region kernels, the 2-D tiled patch
    regulariser as ONE bf16 U-Net call over every tile, Adam + clamp + metrics).  Random-init U-Net
    (reference architecture), synthetic model; the other ranks' observed shots are zeros (never read on
    this rank).  Also the forward / adjoint alone (HIP events) against their algorithmic bytes, and the
    peak HBM allocated."""
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.ssim import SSIM
    from red_diffeq.utils.synthetic import make_model
    torch.manual_seed(8888)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    nt = a.nt
    ctx = dict(n_grid=nx, nt=nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=nx, ns=ns_total)
    fwi = FWIForward(dict(ctx), dev, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none, shots=(0, nsl))
    vt = torch.from_numpy(make_model("curvefault", nz, nx, seed=8888, batch=1))
    with torch.no_grad():
        y_loc = fwi(v_normalize(vt).to(dev))
    y = torch.zeros(1, ns_total, y_loc.shape[2], y_loc.shape[3], device=dev)
    y[:, :nsl] = y_loc
    del y_loc
    mu = torch.nn.functional.pad(prepare_initial_model(vt, "smoothed", sigma=10.0), (1, 1, 1, 1))
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
    diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                             objective="pred_noise").to(dev)
    net.set_precision("bf16")
    eng = InversionEngine(diff, SSIM(), regularization="diffusion", sigma_x0=1e-4, show_progress=False)

    def run(ts):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.optimize(mu, vt, y, fwi, ts=ts, lr=0.03, reg_lambda=0.75, regularization="diffusion")
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(1)                        # plans, buffers and graph captures outside the timing
    t_w = run(1)
    t_all = run(1 + iters)
    ms = (t_all - t_w) / iters * 1e3
    fwi.check()
    # the time loops alone, HIP events on the stream the kernels are launched on
    plan = fwi._plan(nz, nx, dev)
    sz = plan.sizes(1)
    npad = sz.Hp * sz.Wp
    v_in = v_normalize(vt).to(dev)
    dseis = torch.randn(1, nsl, sz.nrec, plan.ng, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fw, ad = [], []
    for _ in range(2):
        coeffs, vstat = plan.coeffs(v_in, 0)
        ev[0].record()
        seis, hist = plan.forward(coeffs, 1, keep_history=True)
        ev[1].record()
        plan.adjoint(coeffs, hist, dseis, 1)
        ev[2].record()
        torch.cuda.synchronize()
        del hist, seis
        fw.append(ev[0].elapsed_time(ev[1]))
        ad.append(ev[1].elapsed_time(ev[2]))
    plan.status()
    f, d = min(fw), min(ad)
    shot_steps = nsl * nt
    peak_gb = torch.cuda.max_memory_allocated(dev) / 1e9
    info = plan.launch_info(1)
    del eng, diff, net, fwi, plan, y, dseis
    torch.cuda.empty_cache()
    return {"workload": f"configs[4] per-rank share: {nz}x{nx} model ({sz.Hp}x{sz.Wp} padded), {nsl} of {ns_total} "
                        f"shots, nt={nt}, one RED-DiffEq iteration (fwd+adj + 2-D tiled bf16 U-Net regulariser + "
                        "Adam + metrics), one GPU, no all-reduce",
            "ms_per_iter": round(ms, 2), "shot_timesteps_per_s": round(shot_steps / (ms * 1e-3), 1),
            "fwd_ms": round(f, 2), "adj_ms": round(d, 2),
            "fwd_GBps_alg": round(12 * npad * shot_steps / f / 1e6, 1),
            "adj_GBps_alg": round(16 * npad * shot_steps / d / 1e6, 1),
            "fwd_frac_alg": round(12 * npad * shot_steps / f / 1e6 / HBM_PEAK_GBS, 4),
            "adj_frac_alg": round(16 * npad * shot_steps / d / 1e6 / HBM_PEAK_GBS, 4),
            # the wide kernels keep T steps of a region on chip, so their counter traffic is below the
            # algorithmic bytes (adjoint 0.81x, forward 0.63x: profiles/r5/pmc_traffic_k_*_tw_ns16.json)
            # and frac_alg can pass 1.0; the cell-step rate is the figure of merit then
            "fwd_gcell_steps_per_s": round(npad * shot_steps / f / 1e6, 1),
            "adj_gcell_steps_per_s": round(npad * shot_steps / d / 1e6, 1),
            "frac_alg_note": "algorithmic fraction (12 / 16 B per cell-step at 8 TB/s); saturates above 1.0",
            "peak_hbm_allocated_GB": round(peak_gb, 1), "kernels": info}


def launch_ranks(a):
    """--gpus N > 1 without a launcher: run N ranks under torch.distributed.run and exit with their
    status.  Only this process's children touch the GPUs (no exec from a GPU-initialised process)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


def unet_rate(dev, reps=20):
    """The configs[2] loop's U-Net forward (dim 64, 72x72, B = 1, fp32 as the reference), as the loop
    runs it (hipGraph replay): ms, conv TFLOP/s and the fraction of the fp32 MFMA peak."""
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(0)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(dev).eval()
    x = torch.randn(1, 1, 72, 72, device=dev)
    t = torch.tensor([500], device=dev)
    def timed(f):
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    with torch.no_grad():
        # the loop's path: inputs written into the captured forward's static buffers, output read in
        # place (RED_DiffEq._eps_residual); and the module call (input copies + output clone)
        xs, ts = net.graph_io(x.shape, x.device)
        xs.copy_(x)
        ts.copy_(t)
        ms = timed(lambda: net.replay_static(xs, ts))
        ms_call = timed(lambda: net(x, t))
    tfs = UNET_GFLOP_72 / (ms * 1e-3) / 1e3
    return {"workload": "U-Net eps-predictor, dim 64, 72x72, B=1, fp32 (configs[2] loop)", "ms": round(ms, 4),
            "ms_module_call": round(ms_call, 4), "conv_tflops": round(tfs, 2), "peak_tflops": FP32_MFMA_PEAK_TFS,
            "mfma_frac": round(tfs / FP32_MFMA_PEAK_TFS, 4)}


def unet_rate_batched(dev, B=25, reps=10):
    """The U-Net forward at configs/openfwi/red-diffeq.yaml's batch (B = 25 tiles of 72 x 72, fp32):
    ms per forward (module call), conv TFLOP/s and the fraction of the fp32 matrix peak."""
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(0)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(dev).eval()
    x = torch.randn(B, 1, 72, 72, device=dev).clamp(-1, 1)
    t = torch.randint(0, 1000, (B,), device=dev)
    with torch.no_grad():
        for _ in range(2):
            net(x, t)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            net(x, t)
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tfs = B * UNET_GFLOP_72 / (ms * 1e-3) / 1e3
    return {"workload": f"U-Net eps-predictor, dim 64, 72x72, B={B}, fp32 (openfwi yaml batch)", "ms": round(ms, 4),
            "conv_tflops": round(tfs, 2), "mfma_frac": round(tfs / FP32_MFMA_PEAK_TFS, 4)}


def conv_class_rates(dev, reps=10, inner=20):
    """fp32 conv classes of the U-Net at B = 1 (the loop; per-tap k_conv_cc), B = 8 and B = 25 (the
    openfwi yaml batch; the 72 x 72 classes on the halo-staged k_conv3_f32 there): device time per
    launch from a hipGraph of `inner` back-to-back launches (launch gaps included), TFLOP/s and the
    fraction of the fp32 matrix peak."""
    shapes = {"l72_3x3_64to64": (64, 0, 64, 72), "l72_3x3_cat128to64": (64, 64, 64, 72),
              "l9_3x3_512to512": (512, 0, 512, 9)}
    out = {}
    for name, (c1, c2, co, H) in shapes.items():
        for B in (1, 8, 25):
            g = torch.Generator(device=dev).manual_seed(0)
            x = torch.randn(B, c1, H, H, device=dev, generator=g)
            x2 = torch.randn(B, c2, H, H, device=dev, generator=g) if c2 else None
            w = torch.randn(co, c1 + c2, 3, 3, device=dev, generator=g) * 0.05
            b = torch.randn(co, device=dev, generator=g)
            f = lambda: torch.ops.red_diffeq.conv2d_mfma(x, x2, w, b, None, 1, 0, False)  # noqa: E731
            for _ in range(2):
                f()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(inner):
                    f()
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                gr.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (reps * inner)
            tf = 2.0 * B * H * H * co * (c1 + c2) * 9 / us / 1e6
            out[f"{name}_B{B}"] = {"us": round(us, 2), "tflops": round(tf, 1), "mfma_frac": round(tf / FP32_MFMA_PEAK_TFS, 3)}
    return out


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RDQ_BENCH_BACKEND=gloo: rehearsal of the N-rank path on a box with fewer GPUs than ranks (ranks
    # share devices round-robin; RCCL needs one GPU per rank).  The driver's runs use RCCL.
    backend = os.environ.get("RDQ_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    # under a torch.distributed launcher the process group is started at every world size, so a
    # world-size-1 torchrun exercises the same init_process_group("nccl", device_id=...) and gradient
    # all-reduce as the N-GPU runs (the driver's plain `python bench.py` N = 1 run has no group)
    distributed = "WORLD_SIZE" in os.environ and "RANK" in os.environ
    if distributed:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    from red_diffeq.core.fused import CosineLR, FusedAdamClamp
    from red_diffeq.core.inversion import grad_all_reduce
    from red_diffeq.core.losses import l1_misfit
    from red_diffeq.regularization.benchmark import total_variation_loss
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.synthetic import make_model

    # N = 1: configs[1] (FlatVel-A, 8 shots).  N > 1: configs[3]'s shape (CurveFault-B, 32 shots per GPU,
    # 256 shots at N = 8), weak scaling; its one-GPU rank workload is reported by the N = 1 line too
    # ("configs3_rank_workload") so a scaling curve can be read on the same per-rank shape.
    nsl = a.ns if a.ns is not None else (8 if world == 1 else 32)
    family = a.family or ("flatvel" if world == 1 else "curvefault")
    B, nt = a.batch, a.nt
    ns_tot = nsl * world
    ctx = dict(n_grid=70, nt=nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=ns_tot)
    fwi = FWIForward(dict(ctx), dev, normalize=True, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none,
                     shots=(rank * nsl, (rank + 1) * nsl))
    if backend != "nccl" and world > torch.cuda.device_count():
        # ranks share a GPU in the rehearsal: whole-chip persistent grids of two processes cannot be
        # co-resident (they would report "not resident"), so the rehearsal runs the chunked kernels
        fwi._plan(70, 70, dev).set_persistent(False)
    vtrue = make_model(family, 70, 70, seed=8888, batch=B)
    vt = torch.from_numpy(vtrue)
    with torch.no_grad():
        y = fwi(v_normalize(vt).to(dev))                         # observed data, local shots
    mu0 = torch.cat([prepare_initial_model(vt[i:i + 1], "smoothed", sigma=10.0) for i in range(B)])
    mu = torch.nn.functional.pad(mu0, (1, 1, 1, 1)).to(dev).requires_grad_(True)
    opt = FusedAdamClamp(mu, lr=0.03, clamp=(-1.0, 1.0))       # K11: Adam + clamp, one pass
    sched = CosineLR(0.03, T_max=300, eta_min=0.0)
    nobs = torch.full((B,), float(ns_tot * nt * 70), device=dev) if distributed else None
    lam = 0.01

    def step():
        v_in = mu[:, :, 1:-1, 1:-1]
        if distributed:
            v_in = grad_all_reduce(v_in)
        loss = l1_misfit(fwi(v_in), y, None, nobs) + lam * total_variation_loss(mu)
        opt.zero_grad()
        loss.sum().backward()
        opt.step()                                              # + clamp_(-1, 1)
        opt.lr = sched.step()

    for _ in range(a.warmup):
        step()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if distributed:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    t_step = el.item() / a.steps
    dbg = os.environ.get("RDQ_DEBUG_STATUS")
    if dbg:
        print("after timed loop:", fwi._plan(70, 70, dev).debug_words(), file=sys.stderr, flush=True)
    fwi.check()          # raises if any persistent launch of the timed region gave up a hand-off

    # ---- phase timing with HIP events on the stream the graphs/kernels are launched on ----
    plan = fwi._plan(70, 70, dev)
    sz = plan.sizes(B)
    npad = sz.Hp * sz.Wp
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    fw_ms, adj_ms = [], []
    v_in = mu.detach()[:, :, 1:-1, 1:-1]
    dseis = torch.randn(B, nsl, sz.nrec, plan.ng, device=dev)
    for _ in range(max(3, a.steps // 2)):
        ev[0].record()
        coeffs, vstat = plan.coeffs(v_in, 0)
        seis, hist = plan.forward(coeffs, B, keep_history=True)
        ev[1].record()
        ev[2].record()
        gA, gk, gb = plan.adjoint(coeffs, hist, dseis, B)
        ev[3].record()
        torch.cuda.synchronize()
        fw_ms.append(ev[0].elapsed_time(ev[1]))
        adj_ms.append(ev[2].elapsed_time(ev[3]))
        del hist
    if dbg:
        print("after phases:", plan.debug_words(), file=sys.stderr, flush=True)
    fwi.check()
    fw_ms, adj_ms = float(np.median(fw_ms)), float(np.median(adj_ms))
    allreduce_us = None
    if distributed:   # the one exchange per iteration: all-reduce of the B x 70 x 70 model gradient
        g = torch.randn(B, 1, 70, 70, device=dev)
        ts_ = []
        for _ in range(25):
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dist.all_reduce(g)
            e1.record()
            torch.cuda.synchronize()
            ts_.append(e0.elapsed_time(e1) * 1e3)
        allreduce_us = round(float(np.median(ts_[5:])), 2)
    info = plan.launch_info(B)
    T = info["adj_T"]
    launches = info["adj_launches"]
    if info["adj_persistent"]:
        kname = f"k_adj_pr<{T}>"                 # the whole adjoint time loop of a shot group is ONE launch
    else:
        kname = f"k_adj_tb<{T}>"                 # one launch per T steps
    shot_steps_per_launch = nsl * B * nt / launches
    steps_per_launch = shot_steps_per_launch / (nsl * B)
    adj_launch_us = adj_ms * 1e3 / launches      # event-timed, incl. the launch's memset nodes
    adj_bytes = 16.0 * npad * shot_steps_per_launch     # adjoint 16*Npad B per shot-step
    fwd_bytes = 12.0 * npad * nsl * B
    achieved = adj_bytes / (adj_launch_us * 1e-6) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", f"pmc_traffic_{kname.replace('<', '').replace('>', '')}_ns{nsl}_B{B}.json")
    if os.path.exists(tfile):
        tj = json.load(open(tfile))
        if tj.get("kernel") == kname:
            traffic = tj["traffic_bytes_per_launch"]

    units = world * nsl * nt * B
    out = {
        "metric": METRIC, "value": round(units / t_step, 1), "unit": "shot-timesteps/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": (("configs[1]: OpenFWI FlatVel-A" if (world == 1 and nsl == 8 and family == "flatvel")
                                 else ("configs[3] shape: OpenFWI CurveFault-B" if (nsl == 32 and family == "curvefault")
                                       else f"OpenFWI {family}")) +
                                f" 70x70 (310x310 padded), {nsl} shots/GPU ({ns_tot} total), nt={nt}, "
                                "fwd+adj gradient + TV + Adam step" +
                                (f" + one {'RCCL' if backend == 'nccl' else backend} all-reduce of the model gradient"
                                 if distributed else "")),
                   "global_batch": B, "shots_per_gpu": nsl, "shots_total": ns_tot, "nt": nt,
                   "parallelism": f"shot-parallel x{world}"},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     # the PMC-measured HBM bytes of the same launch over its time: what the memory system
                     # actually moved.  frac counts SURVEY §8d's 16 B per shot-step; a persistent launch keeps
                     # both wavefield levels of every region in VGPRs and its hand-offs in L2, so only the
                     # history stream and the granules reach HBM (traffic ~0.3x the algorithmic bytes) and
                     # frac can exceed frac_physical (and 1.0) without the kernel being bandwidth-bound
                     "frac_physical": (round(traffic / (adj_launch_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                                       if traffic else None),
                     "algorithmic_bytes_per_launch": adj_bytes, "avg_launch_us": round(adj_launch_us, 3),
                     "steps_per_launch": steps_per_launch,
                     # the figure of merit once frac saturates: the adjoint's device time per time step
                     # (all nsl x B shots), and the forward's (coefficients + forward phase)
                     "adj_us_per_timestep": round(adj_launch_us / steps_per_launch, 4),
                     "fwd_us_per_timestep": round(fw_ms * 1e3 / nt, 4),
                     "traffic_source": os.path.relpath(tfile, ROOT) if traffic is not None else None},
        "kernels": info,
        "phases_ms": {"coeffs+forward": round(fw_ms, 3), "adjoint": round(adj_ms, 3),
                      "fwd_GBps_alg": round(fwd_bytes * nt / (fw_ms * 1e-3) / 1e9, 1)},
        "fwd_adj_only_shot_ts_per_s": round(nsl * nt * B / ((fw_ms + adj_ms) * 1e-3), 1),
        "per_rank": {"shots": nsl, "allreduce_us": allreduce_us, "backend": backend if distributed else None,
                     # step time minus the two time-loop phases; the phases are timed in separate
                     # runs after the timed loop, so this can dip below 0 by the kernels' own
                     # launch-to-launch spread (about +-5 %)
                     "step_minus_kernel_phases_ms": round(t_step * 1e3 - fw_ms - adj_ms, 4)},
    }
    if not a.no_loop:
        # per-iteration wallclock of the drop-in loop itself (InversionEngine.optimize with TV,
        # metrics and histories included), the metric's second half
        out["per_iter_fwi_wallclock_ms"] = loop_wallclock(fwi, mu0, vt, y, a, dev, world)
    if world == 1 and a.ns is None and not a.no_red:
        out["configs3_rank_workload"] = rank_workload_rate(dev, a, 32, "curvefault")
    if world == 1 and not a.no_red:
        out["unet"] = unet_rate(dev)
        out["unet"]["conv_classes"] = conv_class_rates(dev)
        out["unet"]["batched_b25"] = unet_rate_batched(dev)
        out["configs2_red_loop"] = {"workload": "configs[2]: OpenFWI CurveVel-A 70x70, 32 shots, full RED-DiffEq "
                                                "loop (fwd+adj + U-Net regulariser + Adam + metrics), random-init U-Net",
                                    "ms_per_iter": red_loop_wallclock(dev, a),
                                    "shot_timesteps_per_s_incl_unet": None}
        r = out["configs2_red_loop"]
        r["shot_timesteps_per_s_incl_unet"] = round(32 * nt / (r["ms_per_iter"] * 1e-3), 1)
        # the one published number for this path: RED-DiffEq on OpenFWI CF, ns=5,
        # 2.25 s/iter on an RTX 3090 (example/example_openfwi.ipynb:657-658), same loop here
        p_ms = red_loop_wallclock(dev, a, ns=5, family="curvefault")
        # configs/openfwi/red-diffeq.yaml as the reference ships it: batch_size 25 (25 models x 5 shots
        # per iteration through the persistent shot groups, a B = 25 U-Net), CurveFault 70x70
        torch.cuda.reset_peak_memory_stats(dev)
        b25 = red_loop_wallclock(dev, a, ns=5, family="curvefault", batch=25)
        out["openfwi_yaml_b25_red_loop"] = {
            "workload": "configs/openfwi/red-diffeq.yaml: RED-DiffEq loop, OpenFWI CurveFault 70x70, batch_size 25 "
                        "(25 models x 5 shots), nt=1000, random-init dim-64 U-Net at B=25", "ms_per_iter": b25,
            "ms_per_model_iter": round(b25 / 25, 4), "shot_timesteps_per_s": round(25 * 5 * nt / (b25 * 1e-3), 1),
            "peak_hbm_allocated_GB": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)}
        out["published_config_red_loop"] = {
            "workload": "RED-DiffEq loop, OpenFWI CurveFault 70x70, ns=5, nt=1000, B=1 (the reference notebook's "
                        "configuration), random-init U-Net", "ms_per_iter": p_ms,
            "reference_ms_per_iter": 2250.0, "reference_hw": "RTX 3090 (BASELINE.md §1)",
            "speedup_vs_reference": round(2250.0 / p_ms, 1)}
    if world == 1 and a.ns is None and not a.no_configs4:
        out["configs4_rank_workload"] = configs4_rank_workload(dev, a)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(ctx, vtrue[:1], a.cpu_sample_shots, a.cpu_sample_reps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
