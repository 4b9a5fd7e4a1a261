"""configs[4] on the HIP path: the Marmousi-scale 500 x 3000 model (740 x 3240 padded grid), 16 shots
per GPU (the 8-way share of the 128-shot survey), the RED regulariser on 2-D 70 x 70 tiles through ONE
batched U-Net call with bf16 convolutions (mixed precision: bf16 operands, fp32 accumulation).

New behaviour: the reference's patched regulariser only tiles width-wise for models <= 70 rows
(regularization/diffusion.py:85-155), so there is no reference output at this size (parity
unpinned); these tests hold the path to its own definition:
* the batched call's per-tile residuals equal per-tile U-Net calls (B = 1) on the same tiles (fp32:
  to 1e-4; bf16: within the bf16 class, since a bf16 network amplifies summation-order differences);
* the blended gradient equals an independent float64 restatement of the blending (product of the two
  axes' 0.5-overlap weights from calculate_patches, normalised by the weight sum);
* bf16 vs fp32 on the same tiles: relative L2 of the regulariser gradient < 2e-2 (measured ~6e-3);
* three RED-DiffEq iterations of the drop-in InversionEngine at nt = 200: everything finite, the
  data misfit decreases after Adam's first (sign) step.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

NZ, NX = 500, 3000


def _diffusion(cuda):
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    from ckpt_weights import synth_param
    from red_diffeq.models.diffusion import GaussianDiffusion, Unet
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
    diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250, objective="pred_noise")
    sd = diff.state_dict()
    diff.load_state_dict({k: (torch.from_numpy(synth_param(k, v.shape)) if k.startswith("model.") else v)
                          for k, v in sd.items()})
    return diff.to(cuda).eval()


def _blend64(gp, H, W, m):
    """float64 restatement of the 2-D blending: tile (i, j) of the calculate_patches windows along
    rows and columns, weight w_row(i) x w_col(j) with 0.5 on each overlap, normalised by the sum."""
    from red_diffeq.regularization.diffusion import calculate_patches

    def axis(n):
        pos, ov = calculate_patches(n, m)
        ws = []
        for i, (a, b) in enumerate(pos):
            w = np.ones(b - a)
            if i > 0:
                w[:ov[i - 1]] = 0.5
            if i < len(pos) - 1:
                w[-ov[i]:] = 0.5
            ws.append(w)
        return pos, ws
    rows, rws = axis(H)
    cols, cws = axis(W)
    acc = np.zeros((H, W))
    wsum = np.zeros((H, W))
    p = 0
    for (r0, r1), wr in zip(rows, rws):
        for (c0, c1), wc in zip(cols, cws):
            w = wr[:, None] * wc[None, :]
            acc[r0:r1, c0:c1] += gp[p] * w
            wsum[r0:r1, c0:c1] += w
            p += 1
    assert p == len(gp)
    return acc / wsum


def test_configs4_tiled_bf16_regulariser(cuda):
    from red_diffeq.regularization.diffusion import RED_DiffEq, tile_plan
    from red_diffeq.utils.diffusion_utils import diffusion_crop, diffusion_pad
    diff = _diffusion(cuda)
    red = RED_DiffEq(diff, sigma_x0=1e-4)
    g = torch.Generator(device=cuda).manual_seed(44)
    mu = (torch.rand(1, 1, NZ + 2, NX + 2, device=cuda, generator=g) * 2 - 1)
    t = torch.tensor([437], device=cuda)
    noise = torch.randn(1, 1, NZ, NX, device=cuda, generator=g)
    tp = tile_plan(NZ, NX, 70, 1, cuda)
    assert tp.P == 344
    out = {}
    sel = sorted(set(range(0, tp.P, 7)) | {tp.P - 1})       # every 7th tile, both edges included
    with torch.no_grad():
        x0 = diffusion_pad(tp.gather(diffusion_crop(mu)))
        nz = diffusion_pad(tp.gather(noise))
        for prec in ("bf16", "fp32"):
            diff.model.set_precision(prec)
            reg, gpm, _ = red.get_reg_loss_patched(mu, t=t, noise=noise)
            gp = diffusion_crop(red._eps_residual(x0, t.repeat(tp.P), nz))          # one batched call
            grad = tp.assemble(gp)
            # batched tiles vs per-tile calls (B = 1)
            worst = 0.0
            for p in sel:
                one = diffusion_crop(red._eps_residual(x0[p:p + 1], t, nz[p:p + 1]))
                worst = max(worst, float((one - gp[p:p + 1]).abs().max() / gp[p:p + 1].abs().max()))
            out[prec] = (reg, gpm, gp, grad, worst)
        diff.model.set_precision("bf16")
        reg, gpm, gp, grad, worst16 = out["bf16"]
        worst32 = out["fp32"][4]
        assert torch.isfinite(gp).all() and torch.isfinite(grad).all()
        # the regulariser's own outputs are the blended field's (mean, mean of field x mu)
        mu_c = diffusion_crop(mu)
        assert torch.equal(grad, out["bf16"][3])
        assert abs(float(gpm[0]) - float(grad.double().mean())) <= 1e-6 * float(grad.abs().double().mean())
        assert abs(float(reg[0]) - float((grad * mu_c).double().mean())) <= 1e-5 * float((grad * mu_c).abs().double().mean())
        # blending vs the float64 restatement
        ref = _blend64(gp[:, 0].double().cpu().numpy(), NZ, NX, 70)
        blend_err = float(np.abs(grad[0, 0].double().cpu().numpy() - ref).max() / np.abs(ref).max())
        g16, g32 = out["bf16"][3], out["fp32"][3]
        rel = float((g16 - g32).norm() / g32.norm())
    rec = {"tiles": tp.P, "fp32_batched_vs_per_tile_max_rel": worst32, "bf16_batched_vs_per_tile_max_rel": worst16,
           "blend_vs_float64_max_rel": blend_err, "bf16_vs_fp32_rel_l2": rel}
    print(json.dumps(rec))
    d = os.environ.get("RDQ_EVIDENCE_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "configs4_tests.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    assert worst32 <= 1e-4, worst32       # fp32: a tile's result does not depend on its batch
    # bf16: a network of bf16-rounded operands amplifies fp32 summation-order differences (the
    # batch's kernel choice) up to the bf16 rounding level (tools/unet_batch_consistency.py:
    # B = 1 / 8 / 40 differ by ~0.9 % max, fp32 by 2.5e-6), so batched vs per-tile is held to the
    # bf16-vs-fp32 class, not to fp32 rounding
    assert worst16 <= 5e-2, worst16
    assert blend_err <= 1e-6, blend_err
    assert rel < 2e-2, rel


def test_configs4_red_iterations(cuda):
    """Three RED-DiffEq iterations at configs[4]'s size (nt = 200 to bound the test's time; the
    bench tool runs nt = 1000): finite model / histories, decreasing data misfit."""
    from red_diffeq.core.inversion import InversionEngine
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
    from red_diffeq.utils.ssim import SSIM
    from red_diffeq.utils.synthetic import make_model
    diff = _diffusion(cuda)
    diff.model.set_precision("bf16")
    ctx = dict(n_grid=NX, nt=200, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=NX, ns=128)
    fwi = FWIForward(dict(ctx), cuda, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none, shots=(0, 16))
    vt = torch.from_numpy(make_model("curvefault", NZ, NX, seed=8888, batch=1))
    with torch.no_grad():
        y = fwi(v_normalize(vt).to(cuda))
    assert torch.isfinite(y).all()
    mu0 = torch.nn.functional.pad(prepare_initial_model(vt, "smoothed", sigma=10.0), (1, 1, 1, 1))
    yfull = torch.zeros(1, 128, y.shape[2], y.shape[3], device=cuda)
    yfull[:, :16] = y
    eng = InversionEngine(diff, SSIM(), regularization="diffusion", sigma_x0=1e-4, show_progress=False)
    torch.manual_seed(0)
    mu, hist = eng.optimize(mu0, vt, yfull, fwi, ts=3, lr=0.03, reg_lambda=0.75, regularization="diffusion")
    mu = mu.detach()
    assert mu.shape == (1, 1, NZ, NX) and torch.isfinite(mu).all()
    obs = np.array(hist[0]["obs_losses"], np.float64)
    print(json.dumps({"obs_losses": obs.tolist(), "rmse": np.array(hist[0]["rmse"], np.float64).tolist()}))
    assert np.isfinite(obs).all() and all(np.isfinite(np.array(hist[0][k], np.float64)).all() for k in hist[0])
    # Adam's first step moves every cell by +-lr (g / |g|): at nt = 200 the smoothed start already
    # fits the early arrivals (obs[0] ~ 2e-6), so the misfit is held to decrease after that step
    assert obs[2] < obs[1], obs
