"""Arithmetic of the U-Net blocks (reference red_diffeq/models/diffusion.py:78-218) on the HIP
kernels of csrc/unet.hip (C ABI include/red_diffeq_unet.h).

Data movement of the reference graph is folded into the kernels: skip concatenation
(torch.cat, diffusion.py:293-299), nearest x2 upsample (79) and 2x2 pixel-unshuffle (82) into the
conv operand gather; bias, residual adds (168, 286, 290, 297) into the conv / RMSNorm epilogues;
the time-conditioned scale/shift (147) and SiLU into GroupNorm.  There is no PyTorch fallback:
CPU tensors raise.
"""
import contextlib
import ctypes
import math

import torch

from .. import _hip

PLAIN, UPSAMPLE2, UNSHUFFLE2 = 0, 1, 2


def _f(t):
    return t.contiguous() if t is not None else None


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


def _bf16_weights(conv, d, stream):
    """bf16 pack of conv.weight ([cout][tap][cin padded to 32]), cached on the module and rebuilt
    when the weight changes (load_state_dict, in-place updates)."""
    w = conv.weight
    key = (w.data_ptr(), w._version, w.device)
    ent = getattr(conv, "_rdq_bf16", None)
    if ent is None or ent[0] != key:
        L = _hip.lib()
        wp = torch.empty(int(L.rdq_conv2d_bf16_wpack_bytes(ctypes.byref(d))), dtype=torch.uint8, device=w.device)
        _hip.check(L.rdq_conv2d_bf16_pack(ctypes.byref(d), _hip.ptr(w.detach().contiguous()), _hip.ptr(wp), stream),
                   "rdq_conv2d_bf16_pack")
        ent = (key, wp)
        conv._rdq_bf16 = ent
    return ent[1]


def conv2d(x, conv, x2=None, mode=PLAIN, residual=None):
    """nn.Conv2d(stride 1, padding conv.padding) of the logical input formed by `mode`.  Under
    precision("bf16") the dense contractions (K = cin*kh*kw >= 64, cout >= 16: every conv but the
    7x7 single-channel stem and the single-channel output) run on the bf16 matrix cores."""
    _hip.require_device(x)
    x = _f(x)
    x2 = _f(x2)
    w = conv.weight
    cout, cin, kh, kw = w.shape
    B = x.shape[0]
    if mode == UPSAMPLE2:
        H, W = x.shape[2] * 2, x.shape[3] * 2
    elif mode == UNSHUFFLE2:
        H, W = x.shape[2] // 2, x.shape[3] // 2
    else:
        H, W = x.shape[2], x.shape[3]
    cin1 = x.shape[1] * (4 if mode == UNSHUFFLE2 else 1)
    cin2 = x2.shape[1] if x2 is not None else 0
    if cin1 + cin2 != cin:
        raise ValueError(f"conv expects {cin} input channels, got {cin1}+{cin2}")
    pad = conv.padding[0] if isinstance(conv.padding, tuple) else int(conv.padding)
    d = _hip.ConvDesc(B=B, cin1=cin1, cin2=cin2, H=H, W=W, cout=cout, kh=kh, kw=kw, pad=pad, in_mode=mode)
    y = torch.empty(B, cout, H, W, device=x.device, dtype=torch.float32)
    res = _f(residual)
    L = _hip.lib()
    if _PREC["mode"] == "bf16" and cin * kh * kw >= 64 and cout >= 16:
        st = _hip.stream_of(x)
        wp = _bf16_weights(conv, d, st)
        nws = int(L.rdq_conv2d_bf16_ws_bytes(ctypes.byref(d)))
        ws = torch.empty(nws, dtype=torch.uint8, device=x.device) if nws else None
        _hip.check(L.rdq_conv2d_bf16(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(wp), _hip.ptr(conv.bias),
                                     _hip.ptr(res), _hip.ptr(y), _hip.ptr(ws), nws, st), "rdq_conv2d_bf16")
        return y
    nws = int(L.rdq_conv2d_ws_bytes(ctypes.byref(d)))
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device) if nws else None
    _hip.check(L.rdq_conv2d(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(w.contiguous()),
                            _hip.ptr(conv.bias), _hip.ptr(res), _hip.ptr(y), _hip.ptr(ws), nws, _hip.stream_of(x)),
               "rdq_conv2d")
    return y


def linear(x, lin, act_in=0, act_out=0):
    """act_out(Linear(act_in(x))); act 1 = SiLU on the input / GELU(erf) on the output."""
    _hip.require_device(x)
    x = _f(x)
    B, fin = x.shape
    fout = lin.weight.shape[0]
    y = torch.empty(B, fout, device=x.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_linear(B, fin, fout, _hip.ptr(x), _hip.ptr(lin.weight), _hip.ptr(lin.bias), act_in,
                                     act_out, _hip.ptr(y), _hip.stream_of(x)), "rdq_linear")
    return y


def sinusoidal(t, dim, theta=10000):
    _hip.require_device(t)
    t = t.to(torch.int64).contiguous()
    y = torch.empty(t.shape[0], dim, device=t.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_sinusoidal_emb(t.shape[0], dim, float(theta), _hip.ptr(t), _hip.ptr(y),
                                             _hip.stream_of(t)), "rdq_sinusoidal_emb")
    return y


def group_norm_affine_silu(x, norm, scale_shift=None):
    """GroupNorm -> x*(scale+1)+shift -> SiLU; scale_shift: (B, 2C) (scale first, as chunk(2))."""
    _hip.require_device(x)
    x = _f(x)
    B, C, H, W = x.shape
    L = _hip.lib()
    ws = torch.empty(max(8, int(L.rdq_group_norm_ws_bytes(B, C, H * W, norm.num_groups))), dtype=torch.uint8,
                     device=x.device)
    y = torch.empty_like(x)
    ss = _f(scale_shift)
    _hip.check(L.rdq_group_norm_silu(B, C, H * W, norm.num_groups, float(norm.eps), _hip.ptr(x), _hip.ptr(norm.weight),
                                     _hip.ptr(norm.bias), _hip.ptr(ss), _hip.ptr(y), _hip.ptr(ws),
                                     _hip.stream_of(x)), "rdq_group_norm_silu")
    return y


def rmsnorm(x, g, residual=None):
    """F.normalize(x, dim=1) * g * sqrt(C) [+ residual]."""
    _hip.require_device(x)
    x = _f(x)
    B, C, H, W = x.shape
    y = torch.empty_like(x)
    _hip.check(_hip.lib().rdq_rmsnorm(B, C, H * W, _hip.ptr(x), _hip.ptr(g), _hip.ptr(_f(residual)), _hip.ptr(y),
                                      _hip.stream_of(x)), "rdq_rmsnorm")
    return y


def linear_attention(x, m):
    """LinearAttention.forward(x) + x (diffusion.py:182-195 and the residual at 286/297)."""
    B, C, H, W = x.shape
    heads = m.heads
    dh = m.to_qkv.weight.shape[0] // (3 * heads)
    xn = rmsnorm(x, m.norm.g)
    qkv = conv2d(xn, m.to_qkv)
    L = _hip.lib()
    ws = torch.empty(int(L.rdq_linear_attention_ws_bytes(B, heads, dh, H * W, m.mem_kv.shape[-1])),
                     dtype=torch.uint8, device=x.device)
    out = torch.empty(B, heads * dh, H, W, device=x.device, dtype=torch.float32)
    _hip.check(L.rdq_linear_attention(B, heads, dh, H * W, m.mem_kv.shape[-1], float(m.scale), _hip.ptr(qkv),
                                      _hip.ptr(m.mem_kv.contiguous()), _hip.ptr(out), _hip.ptr(ws),
                                      _hip.stream_of(x)), "rdq_linear_attention")
    o = conv2d(out, m.to_out[0])
    return rmsnorm(o, m.to_out[1].g, residual=x)


def full_attention(x, m):
    """Attention.forward(x) + x (diffusion.py:209-218 with Attend(flash=False), residual 290)."""
    B, C, H, W = x.shape
    heads = m.heads
    dh = m.to_qkv.weight.shape[0] // (3 * heads)
    xn = rmsnorm(x, m.norm.g)
    qkv = conv2d(xn, m.to_qkv)
    out = torch.empty(B, heads * dh, H, W, device=x.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_full_attention(B, heads, dh, H * W, m.mem_kv.shape[-2], _hip.ptr(qkv),
                                             _hip.ptr(m.mem_kv.contiguous()), _hip.ptr(out), _hip.stream_of(x)),
               "rdq_full_attention")
    return conv2d(out, m.to_out, residual=x)


def red_q_sample(diff, x0, t, eps):
    """q_sample (diffusion.py:516-519) on the fp32 schedule buffers."""
    x0, eps = _f(x0), _f(eps)
    B = x0.shape[0]
    xt = torch.empty_like(x0)
    _hip.check(_hip.lib().rdq_red_q_sample(B, x0[0].numel(), _hip.ptr(diff.sqrt_alphas_cumprod),
                                           _hip.ptr(diff.sqrt_one_minus_alphas_cumprod), _hip.ptr(t), _hip.ptr(x0),
                                           _hip.ptr(eps), _hip.ptr(xt), _hip.stream_of(x0)), "rdq_red_q_sample")
    return xt


def red_epilogue(diff, xt, t, eps_hat, eps):
    """(eps' - eps) with eps' re-derived from the clipped x0 (diffusion.py:393-419)."""
    xt, eps_hat, eps = _f(xt), _f(eps_hat), _f(eps)
    B = xt.shape[0]
    g = torch.empty_like(xt)
    _hip.check(_hip.lib().rdq_red_epilogue(B, xt[0].numel(), _hip.ptr(diff.sqrt_recip_alphas_cumprod),
                                           _hip.ptr(diff.sqrt_recipm1_alphas_cumprod), _hip.ptr(t), _hip.ptr(xt),
                                           _hip.ptr(eps_hat), _hip.ptr(eps), _hip.ptr(g), _hip.stream_of(xt)),
               "rdq_red_epilogue")
    return g


HIP_OPS = {"conv2d", "linear", "sinusoidal", "group_norm_affine_silu", "rmsnorm", "linear_attention",
           "full_attention", "red_q_sample", "red_epilogue"}
del math
