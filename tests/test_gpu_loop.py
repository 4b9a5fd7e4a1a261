"""Serial-tail kernels (csrc/loop.hip, include/red_diffeq_loop.h) vs plain PyTorch fp32 of the
same ops: K11 fused Adam + clamp vs torch.optim.Adam + clamp_ under the cosine schedule
(reference red_diffeq/core/inversion.py:80-90); K12 fused MAE/RMSE/SSIM vs the torch
MetricsCalculator (red_diffeq/core/metrics.py, utils/ssim.py).  fp32 tolerances are stated per
test (different summation order / FMA contraction)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fused_adam_clamp_matches_torch_adam(cuda):
    from red_diffeq.core.fused import CosineLR, FusedAdamClamp
    torch.manual_seed(0)
    p0 = torch.rand(3, 1, 72, 72, device=cuda) * 2 - 1
    a = p0.clone().requires_grad_(True)
    b = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([a], lr=0.03)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=20, eta_min=0.0)
    fopt = FusedAdamClamp(b, lr=0.03)
    fsch = CosineLR(0.03, T_max=20)
    for _ in range(20):
        g = torch.randn_like(p0) * 0.1
        a.grad = g.clone()
        b.grad = g.clone()
        opt.step()
        with torch.no_grad():
            a.data.clamp_(-1, 1)
        sch.step()
        fopt.step()
        fopt.lr = fsch.step()
        assert abs(fopt.lr - opt.param_groups[0]["lr"]) <= 1e-15
    # per-element fp32 rounding (FMA contraction may differ) accumulated over 20 steps
    assert (a.detach() - b.detach()).abs().max().item() < 2e-6


@pytest.mark.parametrize("shape", [(2, 70, 70), (1, 70, 190), (3, 33, 45)])
def test_fused_metrics_match_torch(cuda, shape):
    from red_diffeq.core.fused import metrics
    from red_diffeq.core.metrics import MetricsCalculator
    from red_diffeq.utils.data_trans import v_normalize
    from red_diffeq.utils.ssim import SSIM
    B, H, W = shape
    torch.manual_seed(1)
    mu = torch.rand(B, 1, H + 2, W + 2, device=cuda) * 2 - 1
    vt = 1500 + 3000 * torch.rand(B, 1, H, W, device=cuda)
    view = mu[:, :, 1:-1, 1:-1]
    mae, rmse, ssim = MetricsCalculator(SSIM()).calculate(view, vt)
    out = metrics(view, v_normalize(vt))
    np.testing.assert_allclose(out[0].cpu().numpy(), mae.cpu().numpy(), rtol=2e-6)
    np.testing.assert_allclose(out[1].cpu().numpy(), rmse.cpu().numpy(), rtol=2e-6)
    np.testing.assert_allclose(out[2].cpu().numpy(), ssim.cpu().numpy(), rtol=0, atol=2e-6)
