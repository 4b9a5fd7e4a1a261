"""Arithmetic of the U-Net blocks (reference red_diffeq/models/diffusion.py:78-218).

Every U-Net block calls these functions; they are the seam where the HIP kernels
(csrc/unet.hip: MFMA implicit-GEMM conv, fused GroupNorm-affine-SiLU, attention) replace the
PyTorch formulation.  Functions without a HIP kernel yet use PyTorch ops on the same device;
``HIP_OPS`` lists the ones that run hand-written kernels.
"""
import torch
import torch.nn.functional as F

HIP_OPS = set()


def pixel_unshuffle2(x):
    """einops 'b c (h p1) (w p2) -> b (c p1 p2) h w' with p1 = p2 = 2 (diffusion.py:82)."""
    return F.pixel_unshuffle(x, 2)


def upsample_nearest2(x):
    """nn.Upsample(scale_factor=2, mode='nearest') (diffusion.py:79)."""
    return F.interpolate(x, scale_factor=2, mode="nearest")


def conv2d(x, conv):
    return F.conv2d(x, conv.weight, conv.bias, padding=conv.padding)


def linear(x, lin):
    return F.linear(x, lin.weight, lin.bias)


def group_norm_affine_silu(x, norm, scale_shift=None):
    """GroupNorm -> x*(scale+1)+shift -> SiLU (Block.forward, diffusion.py:142-149)."""
    x = F.group_norm(x, norm.num_groups, norm.weight, norm.bias, norm.eps)
    if scale_shift is not None:
        scale, shift = scale_shift
        x = x * (scale + 1) + shift
    return F.silu(x)


def rmsnorm(x, g):
    """F.normalize(x, dim=1) * g * sqrt(C) (diffusion.py:84-91)."""
    return F.normalize(x, dim=1) * g * x.shape[1] ** 0.5


def linear_attention(x, m):
    """LinearAttention.forward (diffusion.py:182-195): softmax-feature attention with memory kv."""
    b, c, h, w = x.shape
    heads = m.heads
    xn = rmsnorm(x, m.norm.g)
    qkv = F.conv2d(xn, m.to_qkv.weight).chunk(3, dim=1)
    q, k, v = (t.reshape(b, heads, -1, h * w) for t in qkv)
    mk, mv = (t.unsqueeze(0).expand(b, -1, -1, -1) for t in m.mem_kv)
    k = torch.cat((mk, k), dim=-1)
    v = torch.cat((mv, v), dim=-1)
    q = q.softmax(dim=-2) * m.scale
    k = k.softmax(dim=-1)
    context = torch.einsum("bhdn,bhen->bhde", k, v)
    out = torch.einsum("bhde,bhdn->bhen", context, q).reshape(b, -1, h, w)
    out = F.conv2d(out, m.to_out[0].weight, m.to_out[0].bias)
    return rmsnorm(out, m.to_out[1].g)


def full_attention(x, m):
    """Attention.forward (diffusion.py:209-218) with Attend(flash=False):
    softmax(q k^T / sqrt(d)) v over (memory kv + pixels)."""
    b, c, h, w = x.shape
    heads = m.heads
    xn = rmsnorm(x, m.norm.g)
    qkv = F.conv2d(xn, m.to_qkv.weight).chunk(3, dim=1)
    q, k, v = (t.reshape(b, heads, -1, h * w).transpose(-1, -2) for t in qkv)
    mk, mv = (t.unsqueeze(0).expand(b, -1, -1, -1) for t in m.mem_kv)
    k = torch.cat((mk, k), dim=-2)
    v = torch.cat((mv, v), dim=-2)
    scale = q.shape[-1] ** -0.5
    attn = (torch.einsum("bhid,bhjd->bhij", q, k) * scale).softmax(dim=-1)
    out = torch.einsum("bhij,bhjd->bhid", attn, v)
    out = out.transpose(-1, -2).reshape(b, -1, h, w)
    return F.conv2d(out, m.to_out.weight, m.to_out.bias)
