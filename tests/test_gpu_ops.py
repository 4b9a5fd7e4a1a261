"""torch.ops.red_diffeq.* (red_diffeq/ops.py): every custom operator passes torch.library.opcheck
(schema, autograd registration, FakeTensor / meta kernel agreement with the real output, and for
the shape-generic U-Net / loop ops AOT dispatch with dynamic shapes), and the product modules
(FWIForward, the U-Net, the losses) dispatch through them."""
import numpy as np
import pytest
import torch
from torch.library import opcheck

pytestmark = pytest.mark.gpu

FWI_UTILS = ("test_schema", "test_autograd_registration", "test_faketensor")


@pytest.fixture(scope="module")
def fwi_plan(cuda):
    from red_diffeq.solvers.pde import FWIForward
    from red_diffeq.utils.data_trans import s_normalize_none, v_denormalize
    ctx = dict(n_grid=24, nt=160, dx=10.0, dt=0.001, nbc=10, f=15.0, sz=10, gz=10, ng=24, ns=3)
    fwi = FWIForward(ctx, cuda, v_denorm_func=v_denormalize, s_norm_func=s_normalize_none)
    plan = fwi._plan(20, 24, cuda)
    g = torch.Generator().manual_seed(0)
    v = (torch.rand(2, 1, 20, 24, generator=g) * 1.6 - 0.8).to(cuda)
    return fwi, plan, v


def test_fwi_ops_opcheck(cuda, fwi_plan):
    _, plan, v = fwi_plan
    ops = torch.ops.red_diffeq
    opcheck(ops.fwi_coeffs, (v, plan.op_id, 0), test_utils=FWI_UTILS)
    coeffs, vstat = ops.fwi_coeffs(v, plan.op_id, 0)
    opcheck(ops.fwi_forward, (coeffs, plan.op_id, 2, True), test_utils=FWI_UTILS)
    opcheck(ops.fwi_forward, (coeffs, plan.op_id, 2, False), test_utils=FWI_UTILS)
    seis, hist = ops.fwi_forward(coeffs, plan.op_id, 2, True)
    dseis = torch.randn_like(seis)
    opcheck(ops.fwi_adjoint, (coeffs, hist, dseis, plan.op_id, 2), test_utils=FWI_UTILS)
    gA, gk, gb = ops.fwi_adjoint(coeffs, hist, dseis, plan.op_id, 2)
    opcheck(ops.fwi_grad_finalize, (coeffs, vstat, gA, gk, gb, plan.op_id, 2, 0), test_utils=FWI_UTILS)
    opcheck(ops.fwi, (v.clone().requires_grad_(True), plan.op_id, 0, True), test_utils=FWI_UTILS)


def test_fwi_op_autograd_is_the_adjoint(cuda, fwi_plan):
    """torch.ops.red_diffeq.fwi's registered backward == adjoint + finalize called directly, and
    FWIForward dispatches through the operator."""
    fwi, plan, v = fwi_plan
    vv = v.clone().requires_grad_(True)
    seis = fwi(vv)
    w = torch.randn_like(seis)
    (seis * w).sum().backward()
    ops = torch.ops.red_diffeq
    coeffs, vstat = ops.fwi_coeffs(v, plan.op_id, 0)
    s2, hist = ops.fwi_forward(coeffs, plan.op_id, 2, True)
    assert torch.equal(s2, seis.detach())
    gA, gk, gb = ops.fwi_adjoint(coeffs, hist, w, plan.op_id, 2)
    g = ops.fwi_grad_finalize(coeffs, vstat, gA, gk, gb, plan.op_id, 2, 0)
    assert torch.equal(g, vv.grad)
    fwi.check()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        fwi(v)
    assert any(e.name == "red_diffeq::fwi" for e in prof.events())


def test_unet_and_loop_ops_opcheck(cuda):
    import red_diffeq.ops  # noqa: F401  (registers torch.ops.red_diffeq.*; the test may run alone)
    ops = torch.ops.red_diffeq
    g = torch.Generator().manual_seed(1)

    def r(*s):
        return torch.randn(*s, generator=g).to(cuda)
    x, x2 = r(2, 16, 12, 10), r(2, 8, 12, 10)
    w, b, res = r(24, 24, 3, 3) * 0.1, r(24), r(2, 24, 12, 10)
    for bf16 in (False, True):
        opcheck(ops.conv2d_mfma, (x, x2, w, b, res, 1, 0, bf16))
    opcheck(ops.conv2d_mfma, (x, None, r(8, 16, 3, 3), None, None, 1, 1, False))      # upsample
    opcheck(ops.conv2d_mfma, (x, None, r(8, 64, 1, 1), r(8), None, 0, 2, False))       # unshuffle
    wg = r(64, 24, 3, 3) * 0.1
    opcheck(ops.conv2d_gn_silu, (x, x2, wg, r(64), 1, 0, r(64), r(64), r(2, 128), 8, 1e-5, r(2, 64, 12, 10)))
    opcheck(ops.conv2d_gn_silu, (x, x2, wg, None, 1, 0, r(64), r(64), None, 8, 1e-5, None))
    xb = r(64, 64, 36, 36)                               # 648 halo tiles: the bf16 halo-staged conv
    opcheck(ops.conv2d_bf16_gn_silu, (xb, None, r(128, 64, 3, 3) * 0.1, r(128), 1, 0, r(128), r(128), r(64, 256), 8,
                                      1e-5, None))
    xo = r(128, 64, 36, 36)                              # 648 halo tiles at cout 64
    opcheck(ops.conv2d_bf16_gn_silu_out, (xo, r(64, 64, 3, 3) * 0.1, r(64), 1, r(64), r(64), None, 8, 1e-5, xo,
                                          r(1, 64, 1, 1), r(1)))
    xs, xs2 = r(2, 64, 12, 10), r(2, 64, 12, 10)
    opcheck(ops.conv2d_gn_silu_sc, (xs, xs2, r(64, 128, 3, 3) * 0.1, r(64), r(64), r(64), r(2, 128), 8, 1e-5,
                                    r(64, 128, 1, 1), r(64)))
    xr = r(2, 64, 12, 10)
    opcheck(ops.conv2d_rms, (xr, r(1, 64, 1, 1), r(96, 64, 1, 1), None, None))
    opcheck(ops.conv2d_rms, (xr, r(1, 64, 1, 1), r(64, 64, 1, 1), r(64), xr))
    opcheck(ops.gn_silu, (x, r(16), r(16), r(2, 32), 8, 1e-5))
    opcheck(ops.gn_silu, (x, r(16), r(16), None, 8, 1e-5))
    opcheck(ops.rmsnorm, (x, r(1, 16, 1, 1), x))
    opcheck(ops.linear, (r(2, 32), r(64, 32), r(64), 1, 1))
    opcheck(ops.sinusoidal_emb, (torch.tensor([3, 900], device=cuda), 16, 10000.0))
    opcheck(ops.time_mlp, (torch.tensor([3, 900], device=cuda), 16, 10000.0, r(64, 16), r(64), r(64, 64), r(64)))
    opcheck(ops.linear_silu_multi, (r(2, 64), [r(32, 64), r(128, 64)], [r(32), r(128)]))
    tt = torch.tensor([3, 900], device=cuda)
    opcheck(ops.unet_head, (r(2, 1, 12, 10), r(64, 1, 7, 7), r(64), 3, tt, 16, 10000.0, r(64, 16), r(64), r(64, 64),
                            r(64)))
    opcheck(ops.conv2d_gn_silu_lsm, (xs, r(64, 64, 3, 3) * 0.1, r(64), 1, r(64), r(64), 8, 1e-5, xs, r(2, 64),
                                     [r(128, 64), r(40, 64)], [r(128), r(40)], 0))
    opcheck(ops.conv2d_gn_silu_out, (xs, r(64, 64, 3, 3) * 0.1, r(64), 1, r(64), r(64), r(2, 128), 8, 1e-5, xs2,
                                     r(3, 64, 1, 1), r(3)))
    opcheck(ops.linear_attn, (r(2, 3 * 4 * 8, 6, 6), r(2, 4, 8, 4), 4, 8 ** -0.5))
    qkv, mkv = r(2, 3 * 4 * 32, 6, 6), r(2, 4, 32, 4)
    opcheck(ops.linear_attn_block, (qkv, mkv, 4, 32 ** -0.5, r(64, 128, 1, 1) * 0.1, r(64), r(1, 64, 1, 1),
                                    r(2, 64, 6, 6)))
    opcheck(ops.linear_attn_block, (qkv, mkv, 4, 32 ** -0.5, r(256, 128, 1, 1) * 0.1, None, r(1, 256, 1, 1), None))
    opcheck(ops.attn, (r(2, 3 * 2 * 32, 3, 3), r(2, 2, 4, 32), 2))             # dim_head 32 (the U-Net)
    sa, s1 = torch.rand(1000, device=cuda) + 0.1, torch.rand(1000, device=cuda) + 0.1
    t = torch.tensor([5, 700], device=cuda)
    opcheck(ops.red_q_sample, (r(2, 1, 8, 8), t, r(2, 1, 8, 8), sa, s1))
    opcheck(ops.red_eps, (r(2, 1, 8, 8), t, r(2, 1, 8, 8), r(2, 1, 8, 8), sa, s1))
    xt, tq = torch.empty(2, 1, 8, 8, device=cuda), torch.zeros(2, dtype=torch.int64, device=cuda)
    x0q, eq = r(2, 1, 8, 8), r(2, 1, 8, 8)
    opcheck(ops.red_q_sample_into, (x0q, t, eq, sa, s1, xt, tq))
    ops.red_q_sample_into(x0q, t, eq, sa, s1, xt, tq)
    assert torch.equal(xt, ops.red_q_sample(x0q, t, eq, sa, s1)) and torch.equal(tq, t)
    pred, y = r(2, 3, 20, 7), r(2, 3, 20, 7)
    mask = (torch.rand(2, 3, 20, 7, generator=g) > 0.3).float().to(cuda)
    opcheck(ops.l1_misfit, (pred, y, mask))
    opcheck(ops.l1_misfit, (pred, y, None))
    loss, nobs = ops.l1_misfit(pred, y, mask)
    opcheck(ops.l1_misfit_backward, (pred, y, mask, nobs, r(2)))
    mu = r(2, 1, 14, 14)
    for kind in (0, 1):
        opcheck(ops.smooth_reg, (mu, kind))
        opcheck(ops.smooth_reg_backward, (mu, r(2), kind))
    opcheck(ops.metrics, (mu[:, :, 1:-1, 1:-1], r(2, 1, 12, 12)))


def test_unet_dispatches_through_ops(cuda):
    from red_diffeq.models.diffusion import Unet
    net = Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    x = torch.randn(2, 1, 72, 72, device=cuda)
    t = torch.tensor([10, 500], device=cuda)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        y = net(x, t)                 # grad enabled: the eager path (no hipGraph replay)
    names = {e.name for e in prof.events()}
    for op in ("unet_head", "conv2d_mfma", "conv2d_gn_silu", "gn_silu", "rmsnorm", "linear_silu_multi", "linear_attn",
               "attn"):
        assert f"red_diffeq::{op}" in names, op
    with pytest.raises(RuntimeError, match="no backward"):
        y.sum().backward()
    with torch.no_grad():
        assert torch.equal(net(x, t), y.detach())      # graph replay == eager
    assert np.isfinite(y.detach().cpu().numpy()).all()


@pytest.mark.parametrize("B", [1, 3])
def test_unet_fused_edges_match_separate_launches(cuda, B):
    """The U-Net's fused first / last launches (unet_head: init_conv + time MLP; the first block's conv
    with every block's Linear(SiLU(t)); final_res_block's last pass + final_conv) against the
    separate-launch sequence: head and time projections bit for bit, the output within fp32 rounding
    of the 1x1 conv's summation order."""
    from red_diffeq.models import unet_ops
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(0)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    x = torch.randn(B, 1, 72, 72, device=cuda)
    t = torch.randint(0, 1000, (B,), device=cuda)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        y = net(x, t).detach()
    names = {e.name for e in prof.events()}
    for op in ("unet_head", "conv2d_gn_silu_out") + (("conv2d_gn_silu_lsm",) if B <= 2 else ()):
        assert f"red_diffeq::{op}" in names, op
    x0, te = torch.ops.red_diffeq.unet_head(x, net.init_conv.weight, net.init_conv.bias, 3, t, 64, 10000.0,
                                            net.time_mlp[1].weight, net.time_mlp[1].bias, net.time_mlp[3].weight,
                                            net.time_mlp[3].bias)
    assert torch.equal(x0, unet_ops.conv2d(x, net.init_conv))
    assert torch.equal(te, unet_ops.time_mlp(t, net.time_mlp))
    blocks = net._resnet_blocks()
    h, ss = unet_ops.first_block_and_scale_shifts(x0[:2], blocks[0], te[:2], blocks)
    x0, te = x0[:2], te[:2]
    for a, b in zip(ss, unet_ops.resnet_scale_shifts(te, blocks)):
        assert torch.equal(a, b)
    assert torch.equal(h, blocks[0](x0, te, scale_shift=ss[0]))
    unet_ops.FUSED_EDGES = False
    try:
        with torch.no_grad():
            ysep = net._forward(x, t, None)
    finally:
        unet_ops.FUSED_EDGES = True
    err = (y - ysep).abs().max().item() / ysep.abs().max().item()
    assert err < 2e-6, err
    with torch.no_grad():
        assert torch.equal(net(x, t), y)          # graph replay == eager


def test_unet_static_graph_io(cuda):
    """graph_io / replay_static (the RED regulariser's path: x_t and t written into the captured
    forward's static inputs, output read in place) == forward()."""
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(0)
    net = Unet(dim=16, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    x = torch.randn(2, 1, 72, 72, device=cuda)
    t = torch.tensor([7, 901], device=cuda)
    with torch.no_grad():
        y = net(x, t)
        xs, ts = net.graph_io(x.shape, x.device)
        xs.copy_(x)
        ts.copy_(t)
        assert torch.equal(net.replay_static(xs, ts), y)
        assert net.graph_io(x.shape, x.device)[0] is xs            # one graph per shape
    assert net.graph_io(x.shape, x.device) is None                   # grad enabled: eager, no graph


def test_unet_bf16_batched_fused_tail(cuda):
    """bf16 U-Net at a batch that takes the halo-staged conv everywhere at 72 x 72 (the configs[4] tile
    batch form): the fused tail (block2's normalise pass feeding final_conv) and the bf16 Blocks with
    their statistics in the conv epilogue vs the separate-launch tail, within fp32 rounding."""
    from red_diffeq.models import unet_ops
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(5)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval().set_precision("bf16")
    x = torch.randn(27, 1, 72, 72, device=cuda).clamp(-1, 1)
    t = torch.randint(0, 1000, (27,), device=cuda)
    with torch.no_grad(), torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        y = net(x, t)
    names = {e.name for e in prof.events()}
    for op in ("conv2d_bf16_gn_silu", "conv2d_bf16_gn_silu_out"):
        assert f"red_diffeq::{op}" in names, op
    unet_ops.FUSED_EDGES = False
    try:
        with torch.no_grad():
            ysep = net(x, t)
    finally:
        unet_ops.FUSED_EDGES = True
    err = (y - ysep).abs().max().item() / ysep.abs().max().item()
    assert err < 1e-5, err


def test_adam_clamp_op(cuda):
    """K11 as torch.ops.red_diffeq.adam_clamp_ (mutates param / exp_avg / exp_avg_sq): opcheck, and
    one step equals torch.optim.Adam + clamp_ (reference inversion.py:87-91) within fp32 rounding; a
    set guard word makes it a no-op."""
    from red_diffeq import ops
    g = torch.Generator().manual_seed(3)

    def r(*s):
        return torch.randn(*s, generator=g).to(cuda)
    p, gr, m, v = r(2, 1, 9, 9), r(2, 1, 9, 9), r(2, 1, 9, 9) * 0.1, r(2, 1, 9, 9).abs() * 0.01
    opcheck(ops.adam_clamp_, (p.clone(), gr, m.clone(), v.clone(), 0.9, 0.999, 1e-8, -0.03, 0.5, True, -1.0, 1.0,
                              None))
    word = torch.ones(1, dtype=torch.int32, device=cuda)
    opcheck(ops.adam_clamp_, (p.clone(), gr, m.clone(), v.clone(), 0.9, 0.999, 1e-8, -0.03, 0.5, True, -1.0, 1.0,
                              word))
    q = p.clone()
    ops.adam_clamp_(q, gr, m.clone(), v.clone(), 0.9, 0.999, 1e-8, -0.03, 0.5, True, -1.0, 1.0, word)
    assert torch.equal(q, p)                                   # guarded: no-op
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=0.03)
    ref.grad = gr.clone()
    opt.step()
    with torch.no_grad():
        ref.clamp_(-1, 1)
    q, mq, vq = p.clone(), torch.zeros_like(p), torch.zeros_like(p)
    ops.adam_clamp_(q, gr, mq, vq, 0.9, 0.999, 1e-8, -0.03 / (1 - 0.9), (1 - 0.999) ** 0.5, True, -1.0, 1.0, None)
    assert (q - ref.detach()).abs().max().item() <= 1e-6       # torch foreach Adam: same formula, ulp-level order
