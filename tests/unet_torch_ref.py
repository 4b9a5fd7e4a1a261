"""TEST INFRASTRUCTURE: plain PyTorch fp32 reference of the U-Net block arithmetic
(reference red_diffeq/models/diffusion.py:78-218), used only by tests/test_gpu_unet.py to check
the HIP kernels op by op and the whole U-Net (unet_forward below) on the same device."""
import torch
import torch.nn.functional as F

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


def _block(x, blk, scale_shift=None):
    x = conv2d(x, blk.proj)
    return group_norm_affine_silu(x, blk.norm, scale_shift)


def _resnet(x, m, t):
    ss = None
    if m.mlp is not None:
        te = F.linear(F.silu(t), m.mlp[1].weight, m.mlp[1].bias)
        ss = te[:, :, None, None].chunk(2, dim=1)
    h = _block(x, m.block1, ss)
    h = _block(h, m.block2)
    res = conv2d(x, m.res_conv) if isinstance(m.res_conv, torch.nn.Conv2d) else x
    return h + res


def _attn(x, m):
    from red_diffeq.models.diffusion import Attention
    return full_attention(x, m) if isinstance(m, Attention) else linear_attention(x, m)


def _resample(x, m):
    if isinstance(m, torch.nn.Conv2d):
        return conv2d(x, m)
    if isinstance(m[0], torch.nn.Upsample):
        return conv2d(upsample_nearest2(x), m[1])
    return conv2d(pixel_unshuffle2(x), m[1])


def unet_forward(net, x, time):
    """Unet.forward (diffusion.py:273-301) in plain PyTorch, on net's parameters."""
    import math
    x = conv2d(x, net.init_conv)
    r = x.clone()
    sp = net.time_mlp[0]
    half = sp.dim // 2
    emb = math.log(sp.theta) / (half - 1)
    emb = torch.exp(torch.arange(half, device=x.device) * -emb)
    emb = time[:, None] * emb[None, :]
    t = torch.cat((emb.sin(), emb.cos()), dim=-1)
    t = F.linear(t, net.time_mlp[1].weight, net.time_mlp[1].bias)
    t = F.gelu(t)
    t = F.linear(t, net.time_mlp[3].weight, net.time_mlp[3].bias)
    h = []
    for b1, b2, attn, down in net.downs:
        x = _resnet(x, b1, t)
        h.append(x)
        x = _resnet(x, b2, t)
        x = _attn(x, attn) + x
        h.append(x)
        x = _resample(x, down)
    x = _resnet(x, net.mid_block1, t)
    x = _attn(x, net.mid_attn) + x
    x = _resnet(x, net.mid_block2, t)
    for b1, b2, attn, up in net.ups:
        x = torch.cat((x, h.pop()), dim=1)
        x = _resnet(x, b1, t)
        x = torch.cat((x, h.pop()), dim=1)
        x = _resnet(x, b2, t)
        x = _attn(x, attn) + x
        x = _resample(x, up)
    x = torch.cat((x, r), dim=1)
    x = _resnet(x, net.final_res_block, t)
    return conv2d(x, net.final_conv)
