"""DiffusionFWI baseline (red-diffeq_amd/diffusion_bench, reference diffusion_bench/diffusionfwi.py)
on the HIP operators vs the reference's own trajectory (tests/golden/dfwi_small.npz, made by
tests/golden/make_golden.py on the reference, CPU): 4 reverse-diffusion steps, 3 FWI iterations
each, dim-8 U-Net.  fp32 with different summation orders (GPU kernels vs CPU autograd).

The loop restarts Adam at every diffusion step, and Adam's first step is lr * g / (|g| + eps): a
cell whose gradient is near zero moves by +-lr on the SIGN of an fp32-level quantity.  Measured
(tools/dfwi_sensitivity.py on the GPU): scaling eps_hat by 1 +- 1e-7 moves this run's step-2
misfit by 5.5e-3 relative and two cells of the 14 x 14 model by 2 lr (0.062, 0.064), with every
other cell within 1e-3; the U-Net itself is within 1e-6 of the reference on its fixture.  The
reference driven by the oracle operator happens not to sit on such a cell
(tests/golden/repro_floor.json "dfwi_floor").  The later iterations spread the two flips into
their neighbours (27 more cells between 2e-3 and 1e-2).  Bars: per-step metrics within 1e-2
relative; the final model's mean |diff| within 2e-3, at most 2 % of the cells off by more than
1e-2, none by more than 3 lr.  With
grad_smooth the reference smooths in fp64 on the host (scipy): metrics 1e-2, mean |diff| 2e-3."""
import numpy as np
import pytest
import torch

from conftest import ctx_of, load_golden, record_margin

pytestmark = pytest.mark.gpu


def _diffusion(cuda):
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    z = load_golden("unet_dim8")
    net = Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1)
    net.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")})
    return GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                             objective="pred_noise").to(cuda).eval()


@pytest.mark.parametrize("tag,kw", [("base", {}), ("smooth", dict(grad_smooth=1.0))])
def test_diffusionfwi_vs_reference(cuda, tag, kw):
    from diffusion_bench import DiffusionFWI
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
    from red_diffeq.utils.ssim import SSIM
    z = load_golden("dfwi_small")
    ctx = ctx_of(z)
    fwi = FWIForward(dict(ctx), cuda, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    bench = DiffusionFWI(_diffusion(cuda), fwi, SSIM())
    mu, hist = bench.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]),
                              torch.from_numpy(z["y"]).to(cuda), fwi, ts=3, diffusion_ts=4, lr=0.03, **kw)
    h = hist[0]
    # bars ~10x the measured deviation (profiles/r4/margins.jsonl), except the grad_smooth run's data
    # misfit: its smoothed restart-Adam steps move near-zero-gradient cells by +-lr on fp32-level
    # signs (tools/dfwi_sensitivity.py: 5.5e-3 from an eps-hat perturbation of 1e-7; measured 5.7e-3)
    bars = {"base": dict(obs=3e-4, ssim=3e-4, mae=3e-4, rmse=3e-4, mean=1e-5),
            "smooth": dict(obs=1e-2, ssim=4e-4, mae=4e-4, rmse=4e-4, mean=1e-3)}[tag]
    for k in ("obs", "ssim", "mae", "rmse"):
        key = "obs_losses" if k == "obs" else k
        got, ref = np.array(h[key], np.float64), z[tag + "_" + k].astype(np.float64)
        record_margin("diffusionfwi_metric_rel", f"{tag}:{k}", float(np.max(np.abs(got - ref) / np.abs(ref))), bars[k])
        np.testing.assert_allclose(got, ref, rtol=bars[k], err_msg=k)
    d = np.abs(mu.cpu().numpy() - z[tag + "_mu"])
    record_margin("diffusionfwi_mean_abs_model_dev", tag, float(d.mean()), bars["mean"])
    assert d.mean() < bars["mean"], (d.mean(), d.max())
    if tag == "base":
        assert (d > 1e-2).mean() <= 0.02 and d.max() <= 3 * 0.03, ((d > 1e-2).sum(), d.max())


def test_ilvr_fwi_vs_reference(cuda):
    """ILVR_FWI (diffusion_bench/ilvr_fwi.py) with the reference's recorded q_sample noise injected."""
    from diffusion_bench import ILVR_FWI
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
    from red_diffeq.utils.ssim import SSIM
    z = load_golden("ilvr_small")
    ctx = ctx_of(z)
    fwi = FWIForward(dict(ctx), cuda, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    bench = ILVR_FWI(_diffusion(cuda), fwi, SSIM())
    draws = iter(torch.from_numpy(z["noise"]))
    bench.randn_like = lambda t: next(draws).to(t.device)
    mu, hist = bench.optimize(torch.from_numpy(z["mu0"]), torch.from_numpy(z["v_true"]),
                              torch.from_numpy(z["y"]).to(cuda), fwi, ts=3, diffusion_ts=4, lr=0.03, ilvr_weight=0.3)
    h = hist[0]
    for k in ("obs", "ssim", "mae", "rmse"):
        key = "obs_losses" if k == "obs" else k
        got, ref = np.array(h[key], np.float64), z[k].astype(np.float64)
        record_margin("ilvr_metric_rel", k, float(np.max(np.abs(got - ref) / np.abs(ref))), 8e-4)
        np.testing.assert_allclose(got, ref, rtol=8e-4, err_msg=k)        # measured <= 7.7e-5
    record_margin("ilvr_max_abs_model_dev", "", float(np.abs(mu.cpu().numpy() - z["mu"]).max()), 4e-5)
    assert np.abs(mu.cpu().numpy() - z["mu"]).max() < 4e-5                 # measured 4.1e-6
