"""Arithmetic of the U-Net blocks (reference red_diffeq/models/diffusion.py:78-218) on the HIP
kernels of csrc/unet.hip (C ABI include/red_diffeq_unet.h).

Data movement of the reference graph is folded into the kernels: skip concatenation
(torch.cat, diffusion.py:293-299), nearest x2 upsample (79) and 2x2 pixel-unshuffle (82) into the
conv operand gather; bias, residual adds (168, 286, 290, 297) into the conv / RMSNorm epilogues;
the time-conditioned scale/shift (147) and SiLU into GroupNorm.  Every call goes through the
custom operators torch.ops.red_diffeq.* (red_diffeq/ops.py).  There is no PyTorch fallback: CPU
tensors raise.
"""
import contextlib
import math

import torch

from .. import ops  # noqa: F401  (registers torch.ops.red_diffeq.*)

PLAIN, UPSAMPLE2, UNSHUFFLE2 = 0, 1, 2


# Convolution precision of the current U-Net forward ("fp32", the reference's; or "bf16": bf16
# operands with fp32 accumulation, the configs[4] mixed-precision U-Net).  Set by Unet.forward.
_PREC = {"mode": "fp32"}


@contextlib.contextmanager
def precision(mode):
    if mode not in ("fp32", "bf16"):
        raise ValueError(f"unknown U-Net precision {mode!r} (fp32 | bf16)")
    old = _PREC["mode"]
    _PREC["mode"] = mode
    try:
        yield
    finally:
        _PREC["mode"] = old


def conv2d(x, conv, x2=None, mode=PLAIN, residual=None):
    """nn.Conv2d(stride 1, padding conv.padding) of the logical input formed by `mode`.  Under
    precision("bf16") the dense contractions (K = cin*kh*kw >= 64, cout >= 16: every conv but the
    7x7 single-channel stem and the single-channel output) run on the bf16 matrix cores (weights
    packed once per (tensor, version); ops.clear_bf16_packs() after in-place `.data` updates)."""
    pad = conv.padding[0] if isinstance(conv.padding, tuple) else int(conv.padding)
    return torch.ops.red_diffeq.conv2d_mfma(x, x2, conv.weight, conv.bias, residual, pad, mode,
                                            _PREC["mode"] == "bf16")


def linear(x, lin, act_in=0, act_out=0):
    """act_out(Linear(act_in(x))); act 1 = SiLU on the input / GELU(erf) on the output."""
    return torch.ops.red_diffeq.linear(x, lin.weight, lin.bias, act_in, act_out)


def time_mlp(t, seq):
    """Unet.time_mlp = Sequential(SinusoidalPosEmb, Linear, GELU, Linear) in one launch."""
    return torch.ops.red_diffeq.time_mlp(t, seq[0].dim, float(seq[0].theta), seq[1].weight, seq[1].bias,
                                         seq[3].weight, seq[3].bias)


def resnet_scale_shifts(t, blocks):
    """Every ResnetBlock's Linear(SiLU(t)) (B, 2C) in one launch (at most 32 per call)."""
    out = []
    for i in range(0, len(blocks), 32):
        chunk = blocks[i:i + 32]
        out += torch.ops.red_diffeq.linear_silu_multi(t, [b.mlp[1].weight for b in chunk],
                                                      [b.mlp[1].bias for b in chunk])
    return out


# The fused first / last launches of Unet.forward (head, first_block_and_scale_shifts,
# last_block_and_out); False: the separate-launch sequence (tests compare the two)
FUSED_EDGES = True


def head(x, init_conv, time, seq):
    """(init_conv(x), Unet.time_mlp(time)) in ONE launch (rdq_unet_head) where that form applies, else
    the two separate launches.  The stem conv runs in fp32 under either precision (bf16_eligible)."""
    pad = init_conv.padding[0] if isinstance(init_conv.padding, tuple) else int(init_conv.padding)
    if FUSED_EDGES and ops.unet_head_fusable(x, init_conv.weight, seq):
        return torch.ops.red_diffeq.unet_head(x, init_conv.weight, init_conv.bias, pad, time, seq[0].dim,
                                              float(seq[0].theta), seq[1].weight, seq[1].bias, seq[3].weight,
                                              seq[3].bias)
    return conv2d(x, init_conv), time_mlp(time, seq)


def first_block_and_scale_shifts(x, block, t, blocks):
    """(block(x, scale_shift = its Linear(SiLU(t))), [Linear(SiLU(t)) of every block in `blocks`]) for a
    ResnetBlock with an identity shortcut that is blocks[0]: all the time projections are formed as a
    side job of block1's conv launch (rdq_conv2d_gn_silu_lsm).  None where that form does not apply."""
    b1 = block.block1
    # B <= 2: beyond, the side job costs more than its own launch (tools/lsm_ab.py)
    if not FUSED_EDGES or _PREC["mode"] != "fp32" or x.shape[0] > 2 or not blocks or blocks[0] is not block or \
            len(blocks) > 32 or \
            isinstance(block.res_conv, torch.nn.Conv2d) or any(b.mlp is None for b in blocks):
        return None
    pad = b1.proj.padding[0] if isinstance(b1.proj.padding, tuple) else int(b1.proj.padding)
    if not ops.conv_gn_fusable(x, None, b1.proj.weight, pad, PLAIN, b1.norm.num_groups):
        return None
    h, ss = torch.ops.red_diffeq.conv2d_gn_silu_lsm(
        x, b1.proj.weight, b1.proj.bias, pad, b1.norm.weight, b1.norm.bias, b1.norm.num_groups, float(b1.norm.eps),
        None, t, [b.mlp[1].weight for b in blocks], [b.mlp[1].bias for b in blocks], 0)
    return block.block2(h, post=x), ss


def last_block_and_out(x, block, scale_shift, skip, out_conv):
    """out_conv(block(x, skip, scale_shift)) for a ResnetBlock with a 1x1 shortcut followed by a 1x1
    conv to <= 4 channels (final_res_block + final_conv): block2's normalise pass feeds out_conv
    directly (rdq_conv2d_gn_silu_out; under bf16 rdq_conv2d_bf16_gn_silu_out on the halo-staged conv).
    None where that form does not apply."""
    b2 = block.block2
    if not FUSED_EDGES or out_conv.weight.shape[-1] != 1 or out_conv.weight.shape[0] > 4 or \
            b2.proj.weight.shape[0] % 4 or not isinstance(block.res_conv, torch.nn.Conv2d):
        return None
    pad = b2.proj.padding[0] if isinstance(b2.proj.padding, tuple) else int(b2.proj.padding)
    hshape = (x.shape[0], b2.proj.weight.shape[1], x.shape[2], x.shape[3])
    meta = torch.empty(hshape, device="meta")
    if _PREC["mode"] == "bf16":
        if not ops.conv_gn_bf16_fusable(meta, None, b2.proj.weight, pad, PLAIN, b2.norm.num_groups):
            return None
        h = block.block1(x, scale_shift=scale_shift, skip=skip)
        ys = conv2d(x, block.res_conv, x2=skip)
        return torch.ops.red_diffeq.conv2d_bf16_gn_silu_out(h, b2.proj.weight, b2.proj.bias, pad, b2.norm.weight,
                                                            b2.norm.bias, None, b2.norm.num_groups, float(b2.norm.eps),
                                                            ys, out_conv.weight, out_conv.bias)
    if not ops.conv_gn_fusable(meta, None, b2.proj.weight, pad, PLAIN, b2.norm.num_groups):
        return None
    pair = conv_group_norm_silu_shortcut(x, block.block1.proj, block.block1.norm, scale_shift, skip, block.res_conv)
    if pair is None:
        return None
    return torch.ops.red_diffeq.conv2d_gn_silu_out(pair[0], b2.proj.weight, b2.proj.bias, pad, b2.norm.weight,
                                                   b2.norm.bias, None, b2.norm.num_groups, float(b2.norm.eps), pair[1],
                                                   out_conv.weight, out_conv.bias)


def sinusoidal(t, dim, theta=10000):
    return torch.ops.red_diffeq.sinusoidal_emb(t, dim, float(theta))


def conv_group_norm_silu(x, conv, norm, scale_shift=None, skip=None, post=None):
    """Block.forward: SiLU(GroupNorm(conv(cat(x, skip))) * (scale + 1) + shift) [+ post]; the fused
    two-launch form (statistics in the conv epilogue) where it applies in fp32, else conv +
    GroupNorm (+ add)."""
    pad = conv.padding[0] if isinstance(conv.padding, tuple) else int(conv.padding)
    if _PREC["mode"] == "fp32" and ops.conv_gn_fusable(x, skip, conv.weight, pad, PLAIN, norm.num_groups):
        return torch.ops.red_diffeq.conv2d_gn_silu(x, skip, conv.weight, conv.bias, pad, PLAIN, norm.weight,
                                                   norm.bias, scale_shift, norm.num_groups, float(norm.eps), post)
    if _PREC["mode"] == "bf16" and ops.conv_gn_bf16_fusable(x, skip, conv.weight, pad, PLAIN, norm.num_groups):
        return torch.ops.red_diffeq.conv2d_bf16_gn_silu(x, skip, conv.weight, conv.bias, pad, PLAIN, norm.weight,
                                                        norm.bias, scale_shift, norm.num_groups, float(norm.eps), post)
    h = group_norm_affine_silu(conv2d(x, conv, x2=skip), norm, scale_shift)
    return h + post if post is not None else h


def block_pair(x, skip, block1, block2, scale_shift=None, post=None):
    """block2(block1(cat(x, skip), scale_shift)) [+ post] (ResnetBlock, diffusion.py:160-168) in the bf16
    form that hands block1's output to block2 as bf16 channel octets (conv2d_bf16_block_pair: bit-identical
    to the two Block calls); None where that form does not apply (fp32, or shapes outside the fused conv)."""
    if _PREC["mode"] != "bf16":
        return None
    c1, c2 = block1.proj, block2.proj
    if any((cv.padding[0] if isinstance(cv.padding, tuple) else int(cv.padding)) != 1 for cv in (c1, c2)):
        return None
    G = block1.norm.num_groups
    if block2.norm.num_groups != G or c1.weight.shape[0] % 32:
        return None
    hmeta = torch.empty((x.shape[0], c1.weight.shape[0], x.shape[2], x.shape[3]), device="meta")
    if not (ops.conv_gn_bf16_fusable(x, skip, c1.weight, 1, PLAIN, G) and
            ops.conv_gn_bf16_fusable(hmeta, None, c2.weight, 1, PLAIN, G)):
        return None
    return torch.ops.red_diffeq.conv2d_bf16_block_pair(x, skip, c1.weight, c1.bias, block1.norm.weight, block1.norm.bias,
                                                       scale_shift, float(block1.norm.eps), c2.weight, c2.bias,
                                                       block2.norm.weight, block2.norm.bias, float(block2.norm.eps), G,
                                                       post)


def conv_group_norm_silu_shortcut(x, conv, norm, scale_shift, skip, res_conv):
    """(Block.forward(cat(x, skip)), res_conv(cat(x, skip))) of a ResnetBlock with a 1x1 shortcut: both
    convs in one launch (rdq_conv2d_gn_silu_sc) where that form applies (fp32), else None."""
    if _PREC["mode"] != "fp32" or not isinstance(res_conv, torch.nn.Conv2d) or \
            not ops.conv_gn_sc_fusable(x, skip, conv.weight, res_conv.weight, norm.num_groups):
        return None
    return torch.ops.red_diffeq.conv2d_gn_silu_sc(x, skip, conv.weight, conv.bias, norm.weight, norm.bias, scale_shift,
                                                  norm.num_groups, float(norm.eps), res_conv.weight, res_conv.bias)


def group_norm_affine_silu(x, norm, scale_shift=None):
    """GroupNorm -> x*(scale+1)+shift -> SiLU; scale_shift: (B, 2C) (scale first, as chunk(2))."""
    return torch.ops.red_diffeq.gn_silu(x, norm.weight, norm.bias, scale_shift, norm.num_groups, float(norm.eps))


def rmsnorm(x, g, residual=None):
    """F.normalize(x, dim=1) * g * sqrt(C) [+ residual]."""
    return torch.ops.red_diffeq.rmsnorm(x, g, residual)


def rms_conv(x, norm, conv):
    """conv(RMSNorm(x)) for the attention blocks' to_qkv: the normalisation in the conv's operand
    gather where that form applies (fp32), else RMSNorm then the conv."""
    if _PREC["mode"] == "fp32" and ops.conv_rms_fusable(x, conv.weight):
        return torch.ops.red_diffeq.conv2d_rms(x, norm.g, conv.weight, conv.bias, None)
    return conv2d(rmsnorm(x, norm.g), conv)


# fp32 LinearAttention in the two-launch form (rdq_linear_attention_f32): True / False force it, None
# (default) takes it for the dim-64 blocks of batches of >= 16 (tools/la_f32_ab.py, one block per
# replayed graph: dim 64 at 72 x 72 B = 25 465 -> 348 us, B = 100 1767 -> 1121 us, 36 x 36 149 -> 131 /
# 487 -> 349 us; slower at B = 1 (47 -> 81 us: the chunk combine and one L1 weight load per fp32 MFMA
# step) and for dim 128 at every batch measured).  Otherwise the three-launch form (rms_conv + context +
# output projection); tests compare the two.
FUSED_LA_F32 = None


def _fused_la_f32(x):
    if FUSED_LA_F32 is not None:
        return FUSED_LA_F32
    return x.shape[1] == 64 and x.shape[0] >= 16


def linear_attention(x, m):
    """LinearAttention.forward(x) + x (diffusion.py:182-195 and the residual at 286/297)."""
    conv = m.to_out[0]
    if _PREC["mode"] == "bf16" and ops.linear_attn_bf16_fusable(x, m.to_qkv.weight, conv.weight, m.heads):
        # the whole block in two launches, qkv and the hidden tensor never written (rdq_linear_attention_bf16)
        return torch.ops.red_diffeq.linear_attn_bf16(x, m.norm.g, m.to_qkv.weight, m.mem_kv, conv.weight, conv.bias,
                                                     m.to_out[1].g, m.heads, float(m.scale))
    if _PREC["mode"] == "fp32" and _fused_la_f32(x) and ops.linear_attn_bf16_fusable(x, m.to_qkv.weight,
                                                                                      conv.weight, m.heads):
        # the same two-launch block on fp32 MFMA (rdq_linear_attention_f32)
        return torch.ops.red_diffeq.linear_attn_f32(x, m.norm.g, m.to_qkv.weight, m.mem_kv, conv.weight, conv.bias,
                                                    m.to_out[1].g, m.heads, float(m.scale))
    qkv = rms_conv(x, m.norm, m.to_qkv)
    if _PREC["mode"] == "fp32" and ops.linear_attn_block_fusable(qkv.shape[1], m.heads, conv.weight.shape[0]):
        # context -> (combine, softmax(q) x context, to_out conv, RMSNorm, + x) in one launch (fp32 only: at
        # the configs[4] tile batch under bf16 it measured 1.32 ms per 72 x 72 block against 0.45 + the bf16
        # to_out conv + RMSNorm)
        return torch.ops.red_diffeq.linear_attn_block(qkv, m.mem_kv, m.heads, float(m.scale), conv.weight,
                                                      conv.bias, m.to_out[1].g, x)
    out = torch.ops.red_diffeq.linear_attn(qkv, m.mem_kv, m.heads, float(m.scale))
    return rmsnorm(conv2d(out, conv), m.to_out[1].g, residual=x)


def full_attention(x, m):
    """Attention.forward(x) + x (diffusion.py:209-218 with Attend(flash=False), residual 290)."""
    qkv = rms_conv(x, m.norm, m.to_qkv)
    out = torch.ops.red_diffeq.attn(qkv, m.mem_kv, m.heads)
    return conv2d(out, m.to_out, residual=x)


def red_q_sample(diff, x0, t, eps):
    """q_sample (diffusion.py:516-519) on the fp32 schedule buffers."""
    return torch.ops.red_diffeq.red_q_sample(x0, t, eps, diff.sqrt_alphas_cumprod, diff.sqrt_one_minus_alphas_cumprod)


def red_q_sample_into(diff, x0, t, eps, xt, t_out):
    """red_q_sample written into xt, with t copied to t_out in the same launch (Unet.graph_io)."""
    torch.ops.red_diffeq.red_q_sample_into(x0, t, eps, diff.sqrt_alphas_cumprod, diff.sqrt_one_minus_alphas_cumprod,
                                           xt, t_out)


def red_epilogue(diff, xt, t, eps_hat, eps):
    """(eps' - eps) with eps' re-derived from the clipped x0 (diffusion.py:393-419)."""
    return torch.ops.red_diffeq.red_eps(xt, t, eps_hat, eps, diff.sqrt_recip_alphas_cumprod,
                                        diff.sqrt_recipm1_alphas_cumprod)


HIP_OPS = {"head", "first_block_and_scale_shifts", "last_block_and_out", "conv2d", "conv_group_norm_silu", "conv_group_norm_silu_shortcut", "block_pair", "linear", "time_mlp", "resnet_scale_shifts", "sinusoidal", "group_norm_affine_silu", "rmsnorm", "linear_attention",
           "full_attention", "red_q_sample", "red_q_sample_into", "red_epilogue"}
del math
