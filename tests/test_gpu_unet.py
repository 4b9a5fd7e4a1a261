"""U-Net HIP kernels (csrc/unet.hip) vs a plain PyTorch fp32 reference of the same op
(tests/unet_torch_ref.py) on the same device, and the whole U-Net / RED regulariser vs the
reference's own outputs (tests/golden/unet_dim8.npz, red_dim8.npz; dim=8, same topology).

Tolerances: fp32 with a different summation order (MFMA k-order vs MIOpen / CPU conv):
per-op max-abs <= 2e-5 x scale; whole U-Net <= 2e-4 relative to the output range.
The reference fixtures are "parity unpinned" at Attend (denoising-diffusion-pytorch 2.1.1 is not
installed; its flash=False math is restated)."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

import unet_torch_ref as R
from conftest import load_golden, record_margin

pytestmark = pytest.mark.gpu


def close(a, b, rel=1e-5, what=""):
    """max |a - b| <= rel x max |b|; the measured ratio is recorded next to the bar (record_margin)."""
    scale = max(b.abs().max().item(), 1e-6)
    err = (a - b).abs().max().item()
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    record_margin(test, what, err / scale, rel)
    assert err <= rel * scale, (err, scale)


@pytest.mark.parametrize("cin,cout,k,H,B", [(1, 8, 7, 72, 2), (16, 16, 3, 36, 1), (64, 128, 3, 9, 2),
                                             (24, 40, 1, 18, 3), (7, 5, 3, 10, 1)])
def test_conv_plain(cuda, cin, cout, k, H, B):
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, padding=k // 2).to(cuda)
    x = torch.randn(B, cin, H, H + 2, device=cuda)
    close(ops.conv2d(x, conv), R.conv2d(x, conv))


def test_conv_concat_residual_upsample_unshuffle(cuda):
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(1)
    conv = nn.Conv2d(48, 32, 3, padding=1).to(cuda)
    a = torch.randn(2, 32, 18, 18, device=cuda)
    b = torch.randn(2, 16, 18, 18, device=cuda)
    res = torch.randn(2, 32, 18, 18, device=cuda)
    close(ops.conv2d(a, conv, x2=b, residual=res), R.conv2d(torch.cat((a, b), 1), conv) + res)
    up = nn.Conv2d(32, 16, 3, padding=1).to(cuda)
    close(ops.conv2d(a, up, mode=ops.UPSAMPLE2), R.conv2d(R.upsample_nearest2(a), up))
    dn = nn.Conv2d(128, 64, 1).to(cuda)
    close(ops.conv2d(a, dn, mode=ops.UNSHUFFLE2), R.conv2d(R.pixel_unshuffle2(a), dn))
    nb = nn.Conv2d(32, 8, 1, bias=False).to(cuda)
    close(ops.conv2d(a, nb), R.conv2d(a, nb))


def _conv_abi(x, x2, conv, mode, res, tickets):
    """rdq_conv2d through the C ABI with (pool window) or without (second launch) arrival tickets."""
    import ctypes
    from red_diffeq import _hip, ops as O
    d, shape = O._conv_desc(x, x2, conv.weight, conv.padding[0], mode)
    L = _hip.lib()
    y = torch.empty(shape, device=x.device)
    nws = int(L.rdq_conv2d_ws_bytes(ctypes.byref(d)))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=x.device)
    tk = O._tickets(x.device, int(L.rdq_conv2d_tickets(ctypes.byref(d)))) if tickets else None
    _hip.check(L.rdq_conv2d(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(conv.weight), _hip.ptr(conv.bias),
                            _hip.ptr(res), _hip.ptr(y), _hip.ptr(ws), nws, tk, _hip.stream_of(x)), "rdq_conv2d")
    return y


# the U-Net's own conv shapes at B = 1 and 2 (channel-chunk kernel k_conv_cc: 3x3 over 8-channel
# chunks, 1x1 over 64-channel chunks, split-K combined in-launch by arrival tickets)
@pytest.mark.parametrize("cin1,cin2,cout,k,H,B,mode", [
    (64, 0, 64, 3, 72, 1, 0), (128, 64, 64, 3, 36, 1, 0), (512, 256, 512, 3, 9, 1, 0), (256, 0, 256, 3, 18, 2, 0),
    (256, 0, 128, 3, 36, 1, 1), (64, 0, 384, 1, 72, 1, 0), (256, 128, 256, 1, 18, 1, 0), (256, 0, 128, 1, 18, 1, 2),
    (512, 0, 512, 3, 9, 1, 0), (768, 0, 1536, 1, 9, 1, 0)])
def test_conv_channel_chunk_tickets(cuda, cin1, cin2, cout, k, H, B, mode):
    from red_diffeq import ops as O
    torch.manual_seed(3)
    conv = nn.Conv2d(cin1 + cin2, cout, k, padding=k // 2).to(cuda)
    conv.weight.data *= 0.5
    xs = H // 2 if mode == 1 else 2 * H if mode == 2 else H
    x = torch.randn(B, cin1 // (4 if mode == 2 else 1), xs, xs, device=cuda)
    x2 = torch.randn(B, cin2, H, H, device=cuda) if cin2 else None
    res = torch.randn(B, cout, H, H, device=cuda)
    a = _conv_abi(x, x2, conv, mode, res, True)
    b = _conv_abi(x, x2, conv, mode, res, False)
    assert torch.equal(a, b)                       # in-launch combine == separate combine, bit for bit
    xin = R.upsample_nearest2(x) if mode == 1 else R.pixel_unshuffle2(x) if mode == 2 else x
    if x2 is not None:
        xin = torch.cat((xin, x2), 1)
    close(a, R.conv2d(xin, conv) + res)
    assert int(O._TICKET_POOL[x.device]["pool"].abs().sum()) == 0     # tickets returned to zero


# Block.forward as two launches (GroupNorm statistics in the conv epilogue, rdq_conv2d_gn_silu) vs
# conv -> F.group_norm -> scale/shift -> SiLU (+ identity shortcut) in torch fp32
@pytest.mark.parametrize("cin1,cin2,cout,H,B,ss,post", [
    (64, 0, 64, 72, 1, True, True), (128, 64, 64, 36, 1, True, False), (512, 256, 512, 9, 1, True, False),
    (256, 0, 256, 18, 2, False, True), (64, 0, 128, 9, 3, True, True), (128, 0, 256, 10, 2, True, False),
    (64, 0, 64, 72, 8, True, True), (64, 64, 64, 72, 8, True, False)])
def test_conv_gn_silu_fused(cuda, cin1, cin2, cout, H, B, ss, post):
    from red_diffeq import ops as O
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(6)
    conv = nn.Conv2d(cin1 + cin2, cout, 3, padding=1).to(cuda)
    norm = nn.GroupNorm(8, cout).to(cuda)
    with torch.no_grad():
        norm.weight.mul_(1 + 0.3 * torch.randn_like(norm.weight))
        norm.bias.add_(0.2 * torch.randn_like(norm.bias))
    x = torch.randn(B, cin1, H, H, device=cuda)
    x2 = torch.randn(B, cin2, H, H, device=cuda) if cin2 else None
    sc = torch.randn(B, 2 * cout, device=cuda) if ss else None
    pr = torch.randn(B, cout, H, H, device=cuda) if post else None
    assert O.conv_gn_fusable(x, x2, conv.weight, 1, 0, 8)
    with torch.no_grad():
        got = ops.conv_group_norm_silu(x, conv, norm, sc, skip=x2, post=pr)
        xin = torch.cat((x, x2), 1) if x2 is not None else x
        ref = R.group_norm_affine_silu(R.conv2d(xin, conv), norm, sc[:, :, None, None].chunk(2, dim=1) if ss else None)
        if post:
            ref = ref + pr
    close(got, ref, rel=1e-5)
    assert int(O._TICKET_POOL[x.device]["pool"].abs().sum()) == 0


# ResnetBlock with a 1x1 shortcut: block1's conv and res_conv in one launch (rdq_conv2d_gn_silu_sc),
# bitwise equal to the separate calls, on the U-Net's up-path / final-block shapes
@pytest.mark.parametrize("cin1,cin2,cout,H,B", [(512, 256, 512, 9, 1), (256, 128, 256, 18, 1), (128, 64, 128, 36, 2),
                                                (64, 64, 64, 72, 1)])
def test_conv_gn_silu_with_shortcut(cuda, cin1, cin2, cout, H, B):
    from red_diffeq import ops as O
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(7)
    conv = nn.Conv2d(cin1 + cin2, cout, 3, padding=1).to(cuda)
    res = nn.Conv2d(cin1 + cin2, cout, 1).to(cuda)
    norm = nn.GroupNorm(8, cout).to(cuda)
    x = torch.randn(B, cin1, H, H, device=cuda)
    x2 = torch.randn(B, cin2, H, H, device=cuda)
    sc = torch.randn(B, 2 * cout, device=cuda)
    assert O.conv_gn_sc_fusable(x, x2, conv.weight, res.weight, 8)
    with torch.no_grad():
        y, ys = ops.conv_group_norm_silu_shortcut(x, conv, norm, sc, x2, res)
        ref_y = ops.conv_group_norm_silu(x, conv, norm, sc, skip=x2)
        ref_s = ops.conv2d(x, res, x2=x2)
        tref = R.conv2d(torch.cat((x, x2), 1), res)
    assert torch.equal(y, ref_y)
    assert torch.equal(ys, ref_s)
    close(ys, tref)
    assert int(O._TICKET_POOL[x.device]["pool"].abs().sum()) == 0


# to_qkv(RMSNorm(x)) with the normalisation in the 1x1 conv's gather vs RMSNorm then conv in torch
@pytest.mark.parametrize("C,cout,H,B", [(64, 384, 72, 1), (128, 384, 36, 2), (512, 384, 9, 1), (256, 64, 18, 3)])
def test_conv_rms_fused(cuda, C, cout, H, B):
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(9)
    conv = nn.Conv2d(C, cout, 1, bias=False).to(cuda)
    g = 1 + 0.3 * torch.randn(1, C, 1, 1, device=cuda)
    x = 2 * torch.randn(B, C, H, H, device=cuda) + 0.3

    class N:
        pass
    nm = N()
    nm.g = g
    with torch.no_grad():
        got = ops.rms_conv(x, nm, conv)
        ref = R.conv2d(R.rmsnorm(x, g), conv)
    close(got, ref, rel=1e-5)


@pytest.mark.parametrize("C,H,ss", [(64, 72, True), (16, 9, False), (128, 18, True)])
def test_group_norm_silu(cuda, C, H, ss):
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(2)
    norm = nn.GroupNorm(8, C).to(cuda)
    with torch.no_grad():
        norm.weight.mul_(1 + 0.3 * torch.randn_like(norm.weight))
        norm.bias.add_(0.2 * torch.randn_like(norm.bias))
    x = 3 * torch.randn(2, C, H, H, device=cuda) + 0.5
    sc = torch.randn(2, 2 * C, device=cuda) if ss else None
    ref_ss = sc[:, :, None, None].chunk(2, dim=1) if ss else None
    close(ops.group_norm_affine_silu(x, norm, sc), R.group_norm_affine_silu(x, norm, ref_ss))


def test_rmsnorm_linear_sinusoidal(cuda):
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(3)
    x = torch.randn(2, 96, 9, 9, device=cuda)
    g = torch.randn(1, 96, 1, 1, device=cuda)
    res = torch.randn_like(x)
    close(ops.rmsnorm(x, g), R.rmsnorm(x, g))
    close(ops.rmsnorm(x, g, residual=res), R.rmsnorm(x, g) + res)
    lin = nn.Linear(64, 256).to(cuda)
    v = torch.randn(3, 64, device=cuda)
    close(ops.linear(v, lin), lin(v))
    close(ops.linear(v, lin, act_out=1), torch.nn.functional.gelu(lin(v)))
    close(ops.linear(v, lin, act_in=1), lin(torch.nn.functional.silu(v)))
    t = torch.tensor([0, 17, 803, 999], device=cuda)
    import math
    half = 32
    emb = math.log(10000) / (half - 1)
    f = torch.exp(torch.arange(half, device=cuda) * -emb)
    ref = torch.cat(((t[:, None] * f).sin(), (t[:, None] * f).cos()), -1)
    close(ops.sinusoidal(t, 64), ref, rel=2e-5)


def test_time_mlp_and_scale_shifts(cuda):
    """Unet.time_mlp in one launch and every ResnetBlock's Linear(SiLU(t)) in one launch vs torch."""
    from red_diffeq.models.diffusion import Unet
    from red_diffeq.models import unet_ops as ops
    import torch.nn.functional as F
    torch.manual_seed(7)
    net = Unet(dim=16, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    t = torch.tensor([0, 17, 803, 999], device=cuda)
    with torch.no_grad():
        te = ops.time_mlp(t, net.time_mlp)
        half = 8
        f = torch.exp(torch.arange(half, device=cuda) * -(math.log(10000) / (half - 1)))
        emb = torch.cat(((t[:, None] * f).sin(), (t[:, None] * f).cos()), -1)
        ref = net.time_mlp[3](F.gelu(net.time_mlp[1](emb)))
        close(te, ref, rel=2e-5)
        blocks = net._resnet_blocks()
        ss = ops.resnet_scale_shifts(te, blocks)
        assert len(ss) == len(blocks) == 19
        for b, s in zip(blocks, ss):
            close(s, b.mlp[1](F.silu(te)))


@pytest.mark.parametrize("B", [45, 130])
def test_time_mlp_and_scale_shifts_batched(cuda, B):
    """The large-batch kernels (B > 16: k_time_mlp_b and the sample-per-lane k_wdot_silu_b, whose
    workgroups take 64 samples: a partial last group at both sizes) give every sample exactly what the
    per-sample launch gives it."""
    from red_diffeq.models.diffusion import Unet
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(8)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    t = torch.randint(0, 1000, (B,), device=cuda)
    blocks = net._resnet_blocks()
    with torch.no_grad():
        te = ops.time_mlp(t, net.time_mlp)
        ss = ops.resnet_scale_shifts(te, blocks)
        for i in sorted(i for i in {0, 7, 8, 31, 32, 44, 63, 64, B - 1} if i < B):
            assert torch.equal(te[i:i + 1], ops.time_mlp(t[i:i + 1], net.time_mlp))
            for a, b in zip(ss, ops.resnet_scale_shifts(te[i:i + 1], blocks)):
                assert torch.equal(a[i:i + 1], b)


# the U-Net's linear-attention blocks (dim 64 at 72 / 36, 128 at 18 / 36, 256 at 18): the fused
# block (rdq_linear_attention_block: 21 chunks at 72 x 72 combined in their own launch, <= 8 in the
# output launch), B = 1 and 2; C = 32 takes the unfused three-op path
@pytest.mark.parametrize("C,H,B", [(64, 72, 2), (64, 72, 1), (64, 36, 1), (128, 18, 2), (128, 36, 1), (256, 18, 1),
                                   (256, 18, 2), (32, 18, 2)])
def test_linear_attention(cuda, C, H, B):
    from red_diffeq.models.diffusion import LinearAttention
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(4)
    m = LinearAttention(C).to(cuda)
    with torch.no_grad():
        m.norm.g.mul_(1 + 0.2 * torch.randn_like(m.norm.g))
        m.to_out[1].g.mul_(1 + 0.2 * torch.randn_like(m.to_out[1].g))
    x = torch.randn(B, C, H, H, device=cuda)
    close(ops.linear_attention(x, m), R.linear_attention(x, m) + x, rel=1e-5)


# the configs[4] batched U-Net's levels (72 / 36 / 18) and ragged pixel counts (10 x 10 = 100, 18 x 18 = 324)
@pytest.mark.parametrize("C,H,B", [(64, 72, 3), (64, 72, 40), (64, 36, 5), (128, 36, 2), (128, 18, 7), (64, 10, 3)])
def test_linear_attention_bf16_fused(cuda, C, H, B):
    """LinearAttention.forward(x) + x in the two-launch bf16 form (rdq_linear_attention_bf16: bf16
    operands, fp32 accumulation) vs the fp32 torch restatement; new behaviour (configs[4] mixed
    precision), so the bar is a bf16-level tolerance on the attention output (the residual excluded),
    recorded next to the unfused bf16 path's deviation on the same inputs."""
    from red_diffeq.models.diffusion import LinearAttention
    from red_diffeq.models import unet_ops as ops
    from red_diffeq import ops as O
    torch.manual_seed(40 + C + H)
    m = LinearAttention(C).to(cuda)
    with torch.no_grad():
        m.norm.g.mul_(1 + 0.2 * torch.randn_like(m.norm.g))
        m.to_out[1].g.mul_(1 + 0.2 * torch.randn_like(m.to_out[1].g))
        m.to_out[0].bias.normal_(0, 0.1)
    x = torch.randn(B, C, H, H, device=cuda)
    assert O.linear_attn_bf16_fusable(x, m.to_qkv.weight, m.to_out[0].weight, m.heads)
    with torch.no_grad():
        ref = R.linear_attention(x.double(), m.double()).float()
        m.float()
        with ops.precision("bf16"):
            got = ops.linear_attention(x, m) - x
            qkv = ops.conv2d(ops.rmsnorm(x, m.norm.g), m.to_qkv)
            unf = ops.rmsnorm(ops.conv2d(torch.ops.red_diffeq.linear_attn(qkv, m.mem_kv, m.heads, float(m.scale)),
                                         m.to_out[0]), m.to_out[1].g)
    scale = ref.abs().max().item()
    record_margin("linear_attention_bf16_unfused_max_rel", f"C={C},H={H},B={B}",
                  (unf - ref).abs().max().item() / scale, 3e-2)
    close(got, ref, rel=3e-2, what="fused bf16 vs fp64")


@pytest.mark.parametrize("C,H,B", [(64, 72, 1), (64, 72, 25), (128, 36, 3), (64, 10, 2)])
def test_linear_attention_f32_fused_vs_unfused(cuda, C, H, B):
    """The fp32 two-launch LinearAttention (rdq_linear_attention_f32) vs the three-launch fp32 path and
    vs the torch restatement: fp32 tolerance (1e-5 of the output range; the summation orders differ)."""
    from red_diffeq.models.diffusion import LinearAttention
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(60 + C + H + B)
    m = LinearAttention(C).to(cuda)
    with torch.no_grad():
        m.norm.g.mul_(1 + 0.2 * torch.randn_like(m.norm.g))
        m.to_out[1].g.mul_(1 + 0.2 * torch.randn_like(m.to_out[1].g))
        m.to_out[0].bias.normal_(0, 0.1)
    x = torch.randn(B, C, H, H, device=cuda)
    with torch.no_grad():
        old = ops.FUSED_LA_F32
        try:
            ops.FUSED_LA_F32 = False
            unf = ops.linear_attention(x, m)
            ops.FUSED_LA_F32 = True
            got = ops.linear_attention(x, m)
        finally:
            ops.FUSED_LA_F32 = old
        ref = R.linear_attention(x, m) + x
    close(got, ref, rel=1e-5, what="fused fp32 vs torch")
    close(got, unf, rel=1e-5, what="fused vs three-launch fp32")


# 9 x 9 (the U-Net's level), 8 x 8 and 16 x 16, B = 1 and 2
@pytest.mark.parametrize("C,H,B", [(256, 9, 2), (512, 9, 1), (256, 8, 1), (128, 16, 1)])
def test_full_attention(cuda, C, H, B):
    from red_diffeq.models.diffusion import Attention
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(5)
    m = Attention(C).to(cuda)
    x = torch.randn(B, C, H, H, device=cuda)
    close(ops.full_attention(x, m), R.full_attention(x, m) + x, rel=1e-5)


def _load_unet(cuda):
    from red_diffeq.models.diffusion import Unet
    z = load_golden("unet_dim8")
    net = Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1)
    net.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")})
    return net.to(cuda).eval(), z


def test_unet_dim8_vs_reference_fixture(cuda):
    net, z = _load_unet(cuda)
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["t"]).to(cuda)
    with torch.no_grad():
        out = net(x, t)
        ref_torch = R.unet_forward(net, x, t)
    ref = torch.from_numpy(z["out"]).to(cuda)
    # bars <= 10x what the kernels measure (9.6e-7 / 1.05e-6 of the output range, profiles/r4/margins.jsonl)
    close(out, ref, rel=1e-5, what="vs reference fixture")      # vs the reference implementation (CPU)
    close(out, ref_torch, rel=1e-5, what="vs torch fp32")       # vs plain PyTorch fp32 on the same GPU


@pytest.mark.parametrize("tag", ["sq", "sqw", "patch"])
def test_red_regulariser_vs_reference(cuda, tag):
    from red_diffeq.models.diffusion import GaussianDiffusion
    from red_diffeq.regularization.diffusion import RED_DiffEq
    net, _ = _load_unet(cuda)
    zr = load_golden("red_dim8")
    diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                             objective="pred_noise").to(cuda).eval()
    red = RED_DiffEq(diff, use_time_weight=(tag == "sqw"), sigma_x0=1e-4)
    mu = torch.from_numpy(zr[tag + "_mu"]).to(cuda).requires_grad_(True)
    t = torch.from_numpy(zr[tag + "_t"]).to(cuda)
    noise = torch.from_numpy(zr[tag + "_noise"]).to(cuda)
    fn = red.get_reg_loss_patched if tag == "patch" else red.get_reg_loss
    reg, gpm, tt = fn(mu, t=t, noise=noise)
    reg.sum().backward()
    # measured <= 1.3e-6 of each output's range (profiles/r4/margins.jsonl)
    close(reg.detach(), torch.from_numpy(zr[tag + "_reg"]).to(cuda), rel=1e-5, what="reg")
    close(gpm.detach(), torch.from_numpy(zr[tag + "_gpm"]).to(cuda), rel=1e-5, what="gpm")
    close(mu.grad, torch.from_numpy(zr[tag + "_grad"]).to(cuda), rel=1e-5, what="grad")


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


@pytest.mark.parametrize("cin,cout,k,H,B", [(64, 64, 3, 72, 2), (128, 256, 3, 18, 3), (48, 40, 3, 9, 1),
                                             (256, 128, 1, 9, 2), (512, 512, 3, 9, 1)])
def test_conv_bf16_vs_torch_on_bf16_operands(cuda, cin, cout, k, H, B):
    """Mixed-precision conv (configs[4]): bf16 operands, fp32 accumulation.  Reference: the fp32 torch
    conv of the bf16-ROUNDED input and weights (products of bf16 values are exact in fp32, so only the
    summation order differs).  Covers channel padding (48 -> 64), cout not a multiple of 32, both
    cout-block widths and the split-K path (512 channels at 9x9, B = 1)."""
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(10)
    conv = nn.Conv2d(cin, cout, k, padding=k // 2).to(cuda)
    x = torch.randn(B, cin, H, H, device=cuda)
    ref = torch.nn.functional.conv2d(_bf(x), _bf(conv.weight), conv.bias, padding=k // 2)
    with ops.precision("bf16"):
        got = ops.conv2d(x, conv)
    close(got, ref, rel=2e-5)


def test_conv_bf16_concat_residual_upsample_unshuffle(cuda):
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(11)
    conv = nn.Conv2d(48, 32, 3, padding=1).to(cuda)
    a = torch.randn(2, 32, 18, 18, device=cuda)
    b = torch.randn(2, 16, 18, 18, device=cuda)
    res = torch.randn(2, 32, 18, 18, device=cuda)
    with ops.precision("bf16"):
        got = ops.conv2d(a, conv, x2=b, residual=res)
        up = nn.Conv2d(32, 16, 3, padding=1).to(cuda)
        got_up = ops.conv2d(a, up, mode=ops.UPSAMPLE2)
        dn = nn.Conv2d(128, 64, 1).to(cuda)
        got_dn = ops.conv2d(a, dn, mode=ops.UNSHUFFLE2)
    F = torch.nn.functional
    close(got, F.conv2d(_bf(torch.cat((a, b), 1)), _bf(conv.weight), conv.bias, padding=1) + res)
    close(got_up, F.conv2d(_bf(R.upsample_nearest2(a)), _bf(up.weight), up.bias, padding=1))
    close(got_dn, F.conv2d(_bf(R.pixel_unshuffle2(a)), _bf(dn.weight), dn.bias))


@pytest.mark.parametrize("cin1,cin2,cout,H,B,mode,res", [
    (64, 0, 64, 72, 26, "plain", False),        # tiles straddle images (5184 % 256 = 64), ragged last tile
    (64, 64, 64, 36, 102, "plain", True),       # concatenated skip + residual (decoder ResNet block)
    (24, 16, 128, 36, 52, "plain", False),      # channel padding inside a chunk (40 -> 64), 2 cout tiles
    (128, 0, 128, 18, 51, "up", False),         # nearest-upsampled input (18 -> 36)
    (256, 256, 512, 9, 203, "plain", True),     # 9 x 9 level: halo of 256 + 20 rows, 8 cout tiles
])
def test_conv3_bf16_halo_staged(cuda, cin1, cin2, cout, H, B, mode, res):
    """The halo-staged 3x3 kernel (batched U-Net sizes, >= 512 tiles of 256 pixels x 64 channels):
    against the fp32 torch conv of the bf16-rounded operands, and against the per-tap bf16 kernel
    (rdq_unet_set_option(RDQ_UNET_OPT_BF16_PER_TAP)) with which it shares the operand rounding."""
    from red_diffeq import _hip
    from red_diffeq.models import unet_ops as ops
    F = torch.nn.functional
    torch.manual_seed(14)
    Hin = H // 2 if mode == "up" else H
    conv = nn.Conv2d(cin1 + cin2, cout, 3, padding=1).to(cuda)
    a = torch.randn(B, cin1, Hin, Hin, device=cuda)
    b = torch.randn(B, cin2, H, H, device=cuda) if cin2 else None
    r = torch.randn(B, cout, H, H, device=cuda) if res else None
    md = ops.UPSAMPLE2 if mode == "up" else ops.PLAIN
    with ops.precision("bf16"):
        got = ops.conv2d(a, conv, x2=b, mode=md, residual=r)
        assert _hip.lib().rdq_unet_set_option(1, 1) == 0          # RDQ_UNET_OPT_BF16_PER_TAP
        try:
            per_tap = ops.conv2d(a, conv, x2=b, mode=md, residual=r)
        finally:
            _hip.lib().rdq_unet_set_option(1, 0)
    xin = R.upsample_nearest2(a) if mode == "up" else (torch.cat((a, b), 1) if cin2 else a)
    ref = F.conv2d(_bf(xin), _bf(conv.weight), conv.bias, padding=1) + (r if res else 0)
    close(got, ref, rel=2e-5)
    close(got, per_tap, rel=2e-5)


@pytest.mark.parametrize("cin1,cin2,cout,H,B,mode,res", [
    (64, 0, 64, 72, 10, "plain", False),        # tiles straddle images (5184 % 256 = 64), ragged last tile
    (64, 64, 64, 36, 40, "plain", True),        # concatenated skip + residual (decoder ResNet block)
    (24, 16, 128, 36, 20, "plain", False),      # channel padding inside a 16-channel chunk (40 -> 48)
    (128, 0, 128, 18, 104, "up", False),        # nearest-upsampled input (9 -> 18)
    (256, 256, 512, 9, 80, "plain", True),      # 9 x 9 level: halo of 256 + 20 rows, 8 cout tiles
])
def test_conv3_f32_halo_staged(cuda, cin1, cin2, cout, H, B, mode, res):
    """The fp32 halo-staged 3x3 kernel (k_conv3_f32, >= 192 tiles): against the fp64 conv on the host
    and against the per-tap fp32 kernel (rdq_unet_set_option(RDQ_UNET_OPT_CONV3F_MIN_TILES, 0)):
    exact fp32 products, only the summation order differs."""
    from red_diffeq import _hip
    from red_diffeq.models import unet_ops as ops
    F = torch.nn.functional
    torch.manual_seed(15)
    Hin = H // 2 if mode == "up" else H
    conv = nn.Conv2d(cin1 + cin2, cout, 3, padding=1).to(cuda)
    a = torch.randn(B, cin1, Hin, Hin, device=cuda)
    b = torch.randn(B, cin2, H, H, device=cuda) if cin2 else None
    r = torch.randn(B, cout, H, H, device=cuda) if res else None
    md = ops.UPSAMPLE2 if mode == "up" else ops.PLAIN
    got = ops.conv2d(a, conv, x2=b, mode=md, residual=r)
    old = _hip.lib().rdq_unet_set_option(4, 0)                   # RDQ_UNET_OPT_CONV3F_MIN_TILES
    assert old == 192
    try:
        per_tap = ops.conv2d(a, conv, x2=b, mode=md, residual=r)
    finally:
        _hip.lib().rdq_unet_set_option(4, old)
    xin = R.upsample_nearest2(a) if mode == "up" else (torch.cat((a, b), 1) if cin2 else a)
    ref = F.conv2d(xin.double().cpu(), conv.weight.double().cpu(), conv.bias.double().cpu(), padding=1)
    ref = (ref + (r.double().cpu() if res else 0)).float().to(cuda)
    close(got, ref, rel=5e-6, what="halo fp32 vs fp64")
    close(per_tap, ref, rel=5e-6, what="per-tap fp32 vs fp64")
    close(got, per_tap, rel=5e-6)


def test_unet_fp32_halo_conv_batched(cuda):
    """The fp32 U-Net at the reference's openfwi batch (B = 25: its 72 x 72 and 36 x 36 Blocks, the
    up path's block1 + shortcut and the fused tail on k_conv3_f32, the fused fp32 LinearAttention of
    the dim-64 blocks) against the same network with every conv on the per-tap kernel, and against the
    plain PyTorch fp32 restatement (tests/unet_torch_ref.py; TF32 off)."""
    from red_diffeq import _hip
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(6)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    x = torch.randn(25, 1, 72, 72, device=cuda).clamp(-1, 1)
    t = torch.randint(0, 1000, (25,), device=cuda)
    with torch.no_grad():
        y = net(x, t)
        old = _hip.lib().rdq_unet_set_option(4, 0)
        try:
            net.__dict__.pop("_graphs", None)
            ref = net(x, t)
        finally:
            _hip.lib().rdq_unet_set_option(4, old)
    close(y, ref, rel=2e-5, what="halo vs per-tap network")
    tf32 = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        with torch.no_grad():
            ref_torch = R.unet_forward(net, x, t)
    finally:
        torch.backends.cudnn.allow_tf32 = tf32
    close(y, ref_torch, rel=2e-5, what="vs torch fp32")


# Block.forward on the bf16 halo-staged conv with the GroupNorm statistics in its epilogue
# (rdq_conv2d_bf16_gn_silu, the configs[4] batched U-Net) vs the same conv, its output rounded to bf16
# (the fused path holds the raw conv output as bf16), followed by the separate GroupNorm pass: the
# statistics differ in fp64 summation order only
@pytest.mark.parametrize("cin1,cin2,cout,H,B,ss,post,mode", [
    (64, 0, 64, 72, 32, True, True, "plain"), (64, 64, 64, 72, 32, True, False, "plain"),
    (128, 0, 128, 36, 128, False, True, "plain"), (256, 0, 256, 18, 128, True, False, "plain"),
    (128, 0, 128, 72, 16, True, False, "up")])
def test_conv_bf16_gn_silu_fused(cuda, cin1, cin2, cout, H, B, ss, post, mode):
    from red_diffeq import ops as O
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(21)
    conv = nn.Conv2d(cin1 + cin2, cout, 3, padding=1).to(cuda)
    norm = nn.GroupNorm(8, cout).to(cuda)
    with torch.no_grad():
        norm.weight.mul_(1 + 0.3 * torch.randn_like(norm.weight))
        norm.bias.add_(0.2 * torch.randn_like(norm.bias))
    Hin = H // 2 if mode == "up" else H
    md = ops.UPSAMPLE2 if mode == "up" else ops.PLAIN
    x = torch.randn(B, cin1, Hin, Hin, device=cuda)
    x2 = torch.randn(B, cin2, H, H, device=cuda) if cin2 else None
    sc = torch.randn(B, 2 * cout, device=cuda) if ss else None
    pr = torch.randn(B, cout, H, H, device=cuda) if post else None
    assert O.conv_gn_bf16_fusable(x, x2, conv.weight, 1, md, 8)
    with torch.no_grad(), ops.precision("bf16"):
        got = torch.ops.red_diffeq.conv2d_bf16_gn_silu(x, x2, conv.weight, conv.bias, 1, md, norm.weight, norm.bias,
                                                       sc, 8, float(norm.eps), pr)
        raw = ops.conv2d(x, conv, x2=x2, mode=md).to(torch.bfloat16).float()
        ref = ops.group_norm_affine_silu(raw, norm, sc)
        if post:
            ref = ref + pr
    close(got, ref, rel=1e-5)


# (batches large enough for the halo-staged conv: >= 512 tiles of 256 pixels x 64 channels)
@pytest.mark.parametrize("cin1,cin2,cout,H,B,ss,post", [(64, 0, 64, 72, 26, True, True), (64, 64, 64, 72, 27, True, False),
                                                       (128, 0, 128, 36, 64, False, True), (128, 128, 256, 18, 120, True, False)])
def test_bf16_block_pair_bitexact(cuda, cin1, cin2, cout, H, B, ss, post):
    """ResnetBlock's block1 -> block2 with block1's output handed over as bf16 channel octets
    (conv2d_bf16_block_pair) vs the two Block calls in fp32 storage: bit-identical (block2's conv rounds
    its operands to bf16 either way)."""
    torch.manual_seed(21)
    c1 = nn.Conv2d(cin1 + cin2, cout, 3, padding=1).to(cuda)
    c2 = nn.Conv2d(cout, cout, 3, padding=1).to(cuda)
    n1, n2 = nn.GroupNorm(8, cout).to(cuda), nn.GroupNorm(8, cout).to(cuda)
    with torch.no_grad():
        for n in (n1, n2):
            n.weight.normal_(1, 0.2)
            n.bias.normal_(0, 0.2)
    x = torch.randn(B, cin1, H, H, device=cuda)
    x2 = torch.randn(B, cin2, H, H, device=cuda) if cin2 else None
    sc = torch.randn(B, 2 * cout, device=cuda) * 0.3 if ss else None
    pr = torch.randn(B, cout, H, H, device=cuda) if post else None
    with torch.no_grad():
        got = torch.ops.red_diffeq.conv2d_bf16_block_pair(x, x2, c1.weight, c1.bias, n1.weight, n1.bias, sc, 1e-5,
                                                          c2.weight, c2.bias, n2.weight, n2.bias, 1e-5, 8, pr)
        h = torch.ops.red_diffeq.conv2d_bf16_gn_silu(x, x2, c1.weight, c1.bias, 1, 0, n1.weight, n1.bias, sc, 8, 1e-5,
                                                     None)
        ref = torch.ops.red_diffeq.conv2d_bf16_gn_silu(h, None, c2.weight, c2.bias, 1, 0, n2.weight, n2.bias, None, 8,
                                                       1e-5, pr)
    assert torch.equal(got, ref), (got - ref).abs().max().item()


@pytest.mark.parametrize("B,H,W", [(3, 72, 72), (2, 64, 64), (1, 40, 70), (2, 33, 67)])
def test_stem_direct_conv(cuda, B, H, W):
    """Unet.init_conv (Conv2d(1, 64, 7, padding=3)) under the bf16 precision: the direct fp32 conv
    (rdq_conv2d_stem: two adjacent pixels per thread for even W, a thread per pixel for odd W, all 64
    channels) vs the torch fp32 conv."""
    from red_diffeq.models import unet_ops as ops
    torch.manual_seed(23)
    conv = nn.Conv2d(1, 64, 7, padding=3).to(cuda)
    x = torch.randn(B, 1, H, W, device=cuda)
    with torch.no_grad(), ops.precision("bf16"):
        got = ops.conv2d(x, conv)
    close(got, torch.nn.functional.conv2d(x, conv.weight, conv.bias, padding=3), rel=1e-5)


def test_unet_bf16_close_to_fp32(cuda):
    """Whole U-Net (reference architecture, dim 64) with bf16 convolutions vs fp32: new behaviour
    (configs[4]), no reference counterpart; the deviation is bounded, not bitwise."""
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(12)
    net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    x = torch.randn(6, 1, 72, 72, device=cuda).clamp(-1, 1)
    t = torch.tensor([0, 10, 200, 500, 800, 999], device=cuda)
    with torch.no_grad():
        ref = net(x, t)
        net.set_precision("bf16")
        got = net(x, t)
        net.set_precision("fp32")
        again = net(x, t)
    assert torch.equal(again, ref)
    rel = float((got - ref).norm() / ref.norm())
    record_margin("unet_bf16_vs_fp32_rel_l2", "dim64 B6", rel, 2e-2)
    assert rel < 2e-2, rel


def test_unet_graph_replay_equals_eager(cuda):
    """The hipGraph replay of small no-grad forwards gives the eager result bit for bit, follows
    new inputs, and is re-captured after a weight update."""
    import os
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(13)
    net = Unet(dim=16, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval()
    os.environ["RDQ_NO_UNET_GRAPH"] = "1"
    try:
        xs = [torch.randn(2, 1, 72, 72, device=cuda) for _ in range(2)]
        t = torch.tensor([3, 700], device=cuda)
        with torch.no_grad():
            eager = [net(x, t) for x in xs]
    finally:
        del os.environ["RDQ_NO_UNET_GRAPH"]
    with torch.no_grad():
        got = [net(x, t) for x in xs]
        assert net._graphs, "graph path not taken"
        for a, b in zip(got, eager):
            assert torch.equal(a, b)
        with torch.no_grad():
            net.final_conv.bias.add_(0.5)
        after = net(xs[0], t)
    assert torch.equal(after, eager[0] + 0.5) or (after - eager[0] - 0.5).abs().max() < 1e-6


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_unet_graph_recaptured_after_weights_replaced(cuda, precision):
    """A captured forward must not replay stale weight storage: weights replaced without
    _apply — load_state_dict(assign=True), `p.data = t`, a new nn.Parameter on a submodule — are
    seen by the next no-grad (graph) call, which equals the eager forward of the new weights."""
    import os
    from red_diffeq.models.diffusion import Unet
    torch.manual_seed(15)
    net = Unet(dim=16, dim_mults=(1, 2, 4, 8), channels=1).to(cuda).eval().set_precision(precision)
    x = torch.randn(2, 1, 72, 72, device=cuda)
    t = torch.tensor([5, 600], device=cuda)

    def eager():
        os.environ["RDQ_NO_UNET_GRAPH"] = "1"
        try:
            with torch.no_grad():
                return net(x, t)
        finally:
            del os.environ["RDQ_NO_UNET_GRAPH"]

    with torch.no_grad():
        net(x, t)                                            # captured
        assert net._graphs
        sd = {k: (v * 1.01 if v.is_floating_point() else v).clone() for k, v in net.state_dict().items()}
        net.load_state_dict(sd, assign=True)                 # every parameter on new storage
        got = net(x, t)
        assert torch.equal(got, eager())
        w = net.downs[1][0].block1.proj.weight
        w.data = w.data * 0.9                                 # same Parameter, new storage
        got = net(x, t)
        assert torch.equal(got, eager())
        net.final_conv.weight = nn.Parameter(net.final_conv.weight.detach() * 1.1)   # new Parameter
        got = net(x, t)
        assert torch.equal(got, eager())


def test_post_process_and_p_sample_deterministic_vs_reference(cuda):
    """GaussianDiffusion.p_mean_variance / p_sample_deterministic (reference models/diffusion.py:
    431-452) at t = 0, 37, 640 and RED_DiffEq_POST_PROCESS.diffusion_denoise (regularization/
    diffusion.py:158-200: q_sample to t = 6, six deterministic reverse steps) with the dim-8 U-Net, vs
    the reference's outputs (tests/golden/post_dim8.npz; its randn_like draw replayed)."""
    from red_diffeq.models.diffusion import GaussianDiffusion
    from red_diffeq.regularization.diffusion import RED_DiffEq_POST_PROCESS
    net, _ = _load_unet(cuda)
    z = load_golden("post_dim8")
    diff = GaussianDiffusion(net, image_size=72, timesteps=1000, sampling_timesteps=250,
                             objective="pred_noise").to(cuda).eval()
    x = torch.from_numpy(z["x"]).to(cuda)
    with torch.no_grad():
        for t in (0, 37, 640):
            mean, var, logvar, xs = diff.p_mean_variance(x, torch.full((2,), t, dtype=torch.long, device=cuda))
            close(mean, torch.from_numpy(z[f"pmv{t}_mean"]).to(cuda), rel=2e-5)
            close(xs, torch.from_numpy(z[f"pmv{t}_xs"]).to(cuda), rel=2e-5)
            assert np.allclose(var.reshape(-1).cpu().numpy(), z[f"pmv{t}_var"], rtol=1e-6)
            assert np.allclose(logvar.reshape(-1).cpu().numpy(), z[f"pmv{t}_logvar"], rtol=1e-6)
            m2, xs2 = diff.p_sample_deterministic(x, t)
            assert torch.equal(m2, mean) and torch.equal(xs2, xs)
    noise = torch.from_numpy(z["noise"])
    orig = torch.randn_like
    calls = []

    def replay(t, **kw):
        calls.append(tuple(t.shape))
        return noise.to(t.device)
    torch.randn_like = replay
    try:
        den = RED_DiffEq_POST_PROCESS(diff).diffusion_denoise(torch.from_numpy(z["mu"]).to(cuda), int(z["timesteps"]))
    finally:
        torch.randn_like = orig
    assert calls == [(2, 1, 72, 72)]
    close(den, torch.from_numpy(z["denoised"]).to(cuda), rel=2e-5)
