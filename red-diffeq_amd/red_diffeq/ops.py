"""PyTorch custom operators over the C ABI (torch.ops.red_diffeq.*).

Every HIP entry point the product path uses is registered with torch.library: a schema, the
ROCm implementation (the ctypes call into libred_diffeq_hip.so on the tensor's current stream), a
fake (meta) implementation giving output shapes without running anything, and for the FWI
operator an autograd formula whose backward is the hand-written adjoint.  The ops are
functional (fresh outputs, no input mutation), so torch.library.opcheck, FakeTensor tracing and
torch.compile see them as ordinary operators instead of opaque ctypes calls.

  FWI (include/red_diffeq_fwi.h; a plan is referred to by an integer handle, FwiPlan.op_id)
    red_diffeq::fwi_coeffs(v, plan, vel_mode) -> (coeffs, vstat)                   K3
    red_diffeq::fwi_forward(coeffs, plan, B, keep_history) -> (seis, history)      K1
    red_diffeq::fwi_adjoint(coeffs, history, dseis, plan, B) -> (gA, gk, gbeta)    K2
    red_diffeq::fwi_grad_finalize(coeffs, vstat, gA, gk, gbeta, plan, B, vel_mode) -> grad   K4
    red_diffeq::fwi(v, plan, vel_mode, keep_history) -> (seis, coeffs, vstat, history)
        differentiable in v (register_autograd: adjoint + finalize), what FWIForward calls
  U-Net (include/red_diffeq_unet.h)
    conv2d_mfma, conv2d_rms, conv2d_gn_silu, conv2d_bf16_gn_silu, conv2d_bf16_gn_silu_out, conv2d_gn_silu_sc, conv2d_gn_silu_lsm, conv2d_gn_silu_out, unet_head,
    gn_silu, rmsnorm, linear, time_mlp, linear_silu_multi, sinusoidal_emb, linear_attn, linear_attn_block, attn,
    red_q_sample, red_q_sample_into, red_eps
  loop (include/red_diffeq_loop.h)
    l1_misfit / l1_misfit_backward, smooth_reg / smooth_reg_backward, metrics, adam_clamp_

No CPU implementation is registered: a CPU tensor reaching an op raises (no fallback).
"""
import ctypes
import weakref
from typing import List, Optional, Tuple

import torch
from torch import Tensor
from torch.utils.weak import WeakIdKeyDictionary

from . import _hip

LIB = "red_diffeq"
_PLANS = {}           # op handle -> weakref(FwiPlan); FwiPlan.__del__ unregisters


def register_plan(plan):
    h = id(plan)
    _PLANS[h] = weakref.ref(plan)
    return h


def unregister_plan(h):
    _PLANS.pop(h, None)


def _plan(h):
    ref = _PLANS.get(int(h))
    p = ref() if ref is not None else None
    if p is None:
        raise RuntimeError(f"red_diffeq: unknown FWI plan handle {h}")
    return p


def _f32(n, dev):
    return torch.empty(int(n) // 4, dtype=torch.float32, device=dev)


# ------------------------------------------------------------------------------------------ FWI
@torch.library.custom_op(f"{LIB}::fwi_coeffs", mutates_args=())
def fwi_coeffs(v: Tensor, plan: int, vel_mode: int) -> Tuple[Tensor, Tensor]:
    p = _plan(plan)
    _hip.require_device(v)
    B = v.shape[0]
    sz = p.sizes(B)
    coeffs = _f32(sz.coeffs, v.device)
    vstat = torch.empty(int(sz.vstat), dtype=torch.uint8, device=v.device)
    strides = (ctypes.c_int64 * 4)(*v.stride())
    _hip.check(p.lib.rdq_fwi_coeffs(p.handle, B, _hip.ptr(v), strides, vel_mode, _hip.ptr(coeffs), _hip.ptr(vstat),
                                    _hip.stream_of(v)), "rdq_fwi_coeffs")
    return coeffs, vstat


@fwi_coeffs.register_fake
def _(v, plan, vel_mode):
    sz = _plan(plan).sizes(v.shape[0])
    return (v.new_empty(int(sz.coeffs) // 4, dtype=torch.float32),
            v.new_empty(int(sz.vstat), dtype=torch.uint8))


def _seis_shape(p, B):
    return (B, p.ns, p.sizes(B).nrec, p.ng)


@torch.library.custom_op(f"{LIB}::fwi_forward", mutates_args=())
def fwi_forward(coeffs: Tensor, plan: int, B: int, keep_history: bool) -> Tuple[Tensor, Tensor]:
    p = _plan(plan)
    _hip.require_device(coeffs)
    sz = p.sizes(B)
    seis = torch.empty(_seis_shape(p, B), dtype=torch.float32, device=coeffs.device)
    hist = _f32(sz.history if keep_history else 0, coeffs.device)
    ring = _f32(sz.ring, coeffs.device)
    _hip.check(p.lib.rdq_fwi_forward(p.handle, B, _hip.ptr(coeffs), _hip.ptr(seis),
                                     _hip.ptr(hist) if keep_history else ctypes.c_void_p(0), _hip.ptr(ring),
                                     _hip.stream_of(coeffs)), "rdq_fwi_forward")
    return seis, hist


@fwi_forward.register_fake
def _(coeffs, plan, B, keep_history):
    p = _plan(plan)
    sz = p.sizes(B)
    return (coeffs.new_empty(_seis_shape(p, B)),
            coeffs.new_empty(int(sz.history) // 4 if keep_history else 0))


@torch.library.custom_op(f"{LIB}::fwi_adjoint", mutates_args=())
def fwi_adjoint(coeffs: Tensor, history: Tensor, dseis: Tensor, plan: int, B: int) -> Tuple[Tensor, Tensor, Tensor]:
    p = _plan(plan)
    _hip.require_device(coeffs, history, dseis)
    sz = p.sizes(B)
    if dseis.shape != _seis_shape(p, B) or history.numel() * 4 != sz.history:
        raise ValueError("fwi_adjoint: dseis / history do not match the plan")
    dseis = dseis.float().contiguous()
    ring = _f32(sz.ring, coeffs.device)
    gA = _f32(sz.gA, coeffs.device)
    gk = torch.empty(int(sz.gk_part) // 8, dtype=torch.float64, device=coeffs.device)
    gb = _f32(sz.gbeta, coeffs.device)
    _hip.check(p.lib.rdq_fwi_adjoint(p.handle, B, _hip.ptr(coeffs), _hip.ptr(history), _hip.ptr(dseis),
                                     _hip.ptr(ring), _hip.ptr(gA), _hip.ptr(gk), _hip.ptr(gb),
                                     _hip.stream_of(coeffs)), "rdq_fwi_adjoint")
    return gA, gk, gb


@fwi_adjoint.register_fake
def _(coeffs, history, dseis, plan, B):
    sz = _plan(plan).sizes(B)
    return (coeffs.new_empty(int(sz.gA) // 4), coeffs.new_empty(int(sz.gk_part) // 8, dtype=torch.float64),
            coeffs.new_empty(int(sz.gbeta) // 4))


@torch.library.custom_op(f"{LIB}::fwi_grad_finalize", mutates_args=())
def fwi_grad_finalize(coeffs: Tensor, vstat: Tensor, gA: Tensor, gk: Tensor, gbeta: Tensor, plan: int, B: int,
                      vel_mode: int) -> Tensor:
    p = _plan(plan)
    _hip.require_device(coeffs, gA)
    sz = p.sizes(B)
    colsum = torch.empty(int(sz.colsum) // 8, dtype=torch.float64, device=coeffs.device)
    out = torch.empty(B, 1, p.nz, p.nx, dtype=torch.float32, device=coeffs.device)
    _hip.check(p.lib.rdq_fwi_grad_finalize(p.handle, B, _hip.ptr(coeffs), _hip.ptr(vstat), _hip.ptr(gA), _hip.ptr(gk),
                                           _hip.ptr(gbeta), vel_mode, _hip.ptr(colsum), _hip.ptr(out),
                                           _hip.stream_of(coeffs)), "rdq_fwi_grad_finalize")
    return out


@fwi_grad_finalize.register_fake
def _(coeffs, vstat, gA, gk, gbeta, plan, B, vel_mode):
    p = _plan(plan)
    return coeffs.new_empty(B, 1, p.nz, p.nx)


@torch.library.custom_op(f"{LIB}::fwi", mutates_args=())
def fwi(v: Tensor, plan: int, vel_mode: int, keep_history: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """seis = FWM(v) (K3 + K1); coeffs / vstat / history are returned for the backward."""
    coeffs, vstat = fwi_coeffs(v, plan, vel_mode)
    seis, hist = fwi_forward(coeffs, plan, v.shape[0], keep_history)
    return seis, coeffs, vstat, hist


@fwi.register_fake
def _(v, plan, vel_mode, keep_history):
    coeffs, vstat = _fake_coeffs(v, plan)
    seis, hist = _fake_forward(coeffs, plan, v.shape[0], keep_history)
    return seis, coeffs, vstat, hist


def _fake_coeffs(v, plan):
    sz = _plan(plan).sizes(v.shape[0])
    return v.new_empty(int(sz.coeffs) // 4, dtype=torch.float32), v.new_empty(int(sz.vstat), dtype=torch.uint8)


def _fake_forward(coeffs, plan, B, keep_history):
    p = _plan(plan)
    sz = p.sizes(B)
    return coeffs.new_empty(_seis_shape(p, B)), coeffs.new_empty(int(sz.history) // 4 if keep_history else 0)


def _fwi_setup(ctx, inputs, output):
    v, plan, vel_mode, keep_history = inputs
    _, coeffs, vstat, hist = output
    # only seis is differentiable: no zero "gradients" are materialised for the saved buffers
    # (a zeros_like of the history would be a multi-GB fill per backward)
    ctx.mark_non_differentiable(coeffs, vstat, hist)
    ctx.set_materialize_grads(False)
    if not keep_history:
        ctx.plan = None
        return
    ctx.plan, ctx.vel_mode, ctx.B = plan, vel_mode, v.shape[0]
    ctx.coeffs, ctx.vstat, ctx.hist = coeffs, vstat, hist


def _fwi_backward(ctx, gseis, _gc, _gv, _gh):
    if ctx.plan is None:
        raise RuntimeError("red_diffeq::fwi was called with keep_history=False; no gradient is available")
    gA, gk, gb = fwi_adjoint(ctx.coeffs, ctx.hist, gseis.contiguous(), ctx.plan, ctx.B)
    ctx.hist = None                     # the largest buffer: released as soon as the adjoint has run
    g = fwi_grad_finalize(ctx.coeffs, ctx.vstat, gA, gk, gb, ctx.plan, ctx.B, ctx.vel_mode)
    return g, None, None, None


fwi.register_autograd(_fwi_backward, setup_context=_fwi_setup)


# ---------------------------------------------------------------------------------------- U-Net
# bf16 weight packs, cached per weight TENSOR (weak keys: an entry dies with its tensor, so a new
# tensor at a recycled address never sees a stale pack) and per (version, input split)
_BF16_PACKS = WeakIdKeyDictionary()


def _conv_desc(x, x2, weight, pad, mode):
    cout, cin, kh, kw = weight.shape
    if mode == 1:
        H, W = x.shape[2] * 2, x.shape[3] * 2
    elif mode == 2:
        H, W = x.shape[2] // 2, x.shape[3] // 2
    else:
        H, W = x.shape[2], x.shape[3]
    cin1 = x.shape[1] * (4 if mode == 2 else 1)
    cin2 = x2.shape[1] if x2 is not None else 0
    if cin1 + cin2 != cin:
        raise ValueError(f"conv expects {cin} input channels, got {cin1}+{cin2}")
    return _hip.ConvDesc(B=x.shape[0], cin1=cin1, cin2=cin2, H=H, W=W, cout=cout, kh=kh, kw=kw, pad=pad,
                         in_mode=mode), (x.shape[0], cout, H, W)


def _bf16_pack(weight, d, stream):
    per = _BF16_PACKS.setdefault(weight, {})
    key = (weight._version, weight.data_ptr(), d.cin1, d.cin2)   # data_ptr: `p.data = t` replaces storage
    wp = per.get(key)
    if wp is None:
        per.clear()                      # older versions of this tensor are dead
        L = _hip.lib()
        wp = torch.empty(int(L.rdq_conv2d_bf16_wpack_bytes(ctypes.byref(d))), dtype=torch.uint8, device=weight.device)
        _hip.check(L.rdq_conv2d_bf16_pack(ctypes.byref(d), _hip.ptr(weight.contiguous()), _hip.ptr(wp), stream),
                   "rdq_conv2d_bf16_pack")
        per[key] = wp
    return wp


def clear_bf16_packs():
    """Drop the cached bf16 weight packs: needed after in-place updates through `.data`, which do
    not bump a tensor's version counter."""
    _BF16_PACKS.clear()


def bf16_eligible(weight):
    cout, cin, kh, kw = weight.shape
    return cin * kh * kw >= 64 and cout >= 16


@torch.library.custom_op(f"{LIB}::conv2d_mfma", mutates_args=())
def conv2d_mfma(x: Tensor, x2: Optional[Tensor], weight: Tensor, bias: Optional[Tensor], residual: Optional[Tensor],
                pad: int, mode: int, bf16: bool) -> Tensor:
    """nn.Conv2d (stride 1) of the logical input cat(x', x2), x' = x | upsample2(x) | unshuffle2(x)
    (mode 0 / 1 / 2), + bias + residual; fp32 MFMA, or bf16 operands with fp32 accumulation."""
    _hip.require_device(x)
    x = x.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    d, shape = _conv_desc(x, x2, weight, pad, mode)
    y = torch.empty(shape, device=x.device, dtype=torch.float32)
    res = residual.contiguous() if residual is not None else None
    L = _hip.lib()
    st = _hip.stream_of(x)
    if bf16 and tuple(weight.shape) == (64, 1, 7, 7) and pad == 3 and mode == 0 and x2 is None and residual is None \
            and 64 <= x.shape[3] <= 72:
        # the batched bf16 U-Net's stem (an fp32 conv: K = 49 is below the bf16 floor) as a direct conv
        _hip.check(L.rdq_conv2d_stem(ctypes.byref(d), _hip.ptr(x), _hip.ptr(weight.contiguous()), _hip.ptr(bias),
                                     _hip.ptr(y), st), "rdq_conv2d_stem")
        return y
    if bf16 and bf16_eligible(weight):
        wp = _bf16_pack(weight, d, st)
        nws = int(L.rdq_conv2d_bf16_ws_bytes(ctypes.byref(d)))
        ws = torch.empty(nws, dtype=torch.uint8, device=x.device) if nws else None
        _hip.check(L.rdq_conv2d_bf16(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(wp), _hip.ptr(bias),
                                     _hip.ptr(res), _hip.ptr(y), _hip.ptr(ws), nws, st), "rdq_conv2d_bf16")
        return y
    nws = int(L.rdq_conv2d_ws_bytes(ctypes.byref(d)))
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device) if nws else None
    tk = _tickets(x.device, int(L.rdq_conv2d_tickets(ctypes.byref(d)))) if nws else None
    _hip.check(L.rdq_conv2d(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(weight.contiguous()), _hip.ptr(bias),
                            _hip.ptr(res), _hip.ptr(y), _hip.ptr(ws), nws, tk, st), "rdq_conv2d")
    return y


# Split-K arrival tickets of rdq_conv2d (include/red_diffeq_unet.h): one zeroed pool per device,
# every launch leaves its words zero again.  Eager calls take consecutive windows of a ring (a window
# comes round again only thousands of launches later); calls captured into a hipGraph get windows
# that no later call reuses, since a graph replays with the same words, possibly beside eager work
# on another stream.  No pool yet (first call inside a capture) or the graph region used up: no
# tickets, and the slabs are combined by a second launch instead (same result).
_TICKET_POOL = {}
_TICKET_EAGER, _TICKET_GRAPH = 1 << 18, 1 << 19


def _tickets(device, n):
    capturing = torch.cuda.is_current_stream_capturing()
    st = _TICKET_POOL.get(device)
    if st is None:
        if capturing:
            return None
        st = _TICKET_POOL[device] = {"pool": torch.zeros(_TICKET_EAGER + _TICKET_GRAPH, dtype=torch.int32,
                                                         device=device), "eager": 0, "graph": 0}
    if capturing:
        if st["graph"] + n > _TICKET_GRAPH:
            return None
        off = _TICKET_EAGER + st["graph"]
        st["graph"] += n
    else:
        if st["eager"] + n > _TICKET_EAGER:
            st["eager"] = 0
        off = st["eager"]
        st["eager"] += n
    return st["pool"].data_ptr() + 4 * off


@conv2d_mfma.register_fake
def _(x, x2, weight, bias, residual, pad, mode, bf16):
    _, shape = _conv_desc(x, x2, weight, pad, mode)
    return x.new_empty(shape)


@torch.library.custom_op(f"{LIB}::gn_silu", mutates_args=())
def gn_silu(x: Tensor, weight: Tensor, bias: Tensor, scale_shift: Optional[Tensor], groups: int, eps: float) -> Tensor:
    """GroupNorm(groups) -> x * (scale + 1) + shift -> SiLU; scale_shift (B, 2C), scale first."""
    _hip.require_device(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    L = _hip.lib()
    ws = torch.empty(max(8, int(L.rdq_group_norm_ws_bytes(B, C, H * W, groups))), dtype=torch.uint8, device=x.device)
    y = torch.empty_like(x)
    ss = scale_shift.contiguous() if scale_shift is not None else None
    _hip.check(L.rdq_group_norm_silu(B, C, H * W, groups, float(eps), _hip.ptr(x), _hip.ptr(weight), _hip.ptr(bias),
                                     _hip.ptr(ss), _hip.ptr(y), _hip.ptr(ws), _hip.stream_of(x)), "rdq_group_norm_silu")
    return y


@gn_silu.register_fake
def _(x, weight, bias, scale_shift, groups, eps):
    return torch.empty_like(x)


def conv_rms_fusable(x, weight):
    """rdq_conv2d_rms applies: 1x1 conv, channel counts multiples of 64 (<= 2048), fp32 extents."""
    cout, cin, kh, kw = weight.shape
    return kh == 1 and kw == 1 and cin % 64 == 0 and cin <= 2048 and x.shape[1] == cin and \
        x.numel() * 4 < 2 ** 31 and x.shape[0] * cout * x.shape[2] * x.shape[3] * 4 < 2 ** 31


@torch.library.custom_op(f"{LIB}::conv2d_rms", mutates_args=())
def conv2d_rms(x: Tensor, g: Tensor, weight: Tensor, bias: Optional[Tensor], residual: Optional[Tensor]) -> Tensor:
    """1x1 conv of RMSNorm(x) = F.normalize(x, dim=1) * g * sqrt(C) (the attention blocks' to_qkv,
    diffusion.py:184-186, 211-213), the normalisation formed in the conv's operand gather."""
    _hip.require_device(x)
    x = x.contiguous()
    d, shape = _conv_desc(x, None, weight, 0, 0)
    L = _hip.lib()
    nws = int(L.rdq_conv2d_ws_bytes(ctypes.byref(d)))
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device) if nws else None
    tk = _tickets(x.device, int(L.rdq_conv2d_tickets(ctypes.byref(d)))) if nws else None
    y = torch.empty(shape, device=x.device, dtype=torch.float32)
    res = residual.contiguous() if residual is not None else None
    _hip.check(L.rdq_conv2d_rms(ctypes.byref(d), _hip.ptr(x), _hip.ptr(g.contiguous()), _hip.ptr(weight.contiguous()),
                                _hip.ptr(bias), _hip.ptr(res), _hip.ptr(y), _hip.ptr(ws), nws, tk,
                                _hip.stream_of(x)), "rdq_conv2d_rms")
    return y


@conv2d_rms.register_fake
def _(x, g, weight, bias, residual):
    _, shape = _conv_desc(x, None, weight, 0, 0)
    return x.new_empty(shape)


def conv_gn_fusable(x, x2, weight, pad, mode, groups):
    """rdq_conv2d_gn_silu applies to this conv + GroupNorm (fp32 channel-chunk conv, H*W >= 32,
    C / G in {8, 16, 32, 64})."""
    d, _ = _conv_desc(x, x2, weight, pad, mode)
    return int(_hip.lib().rdq_conv2d_gn_ws_bytes(ctypes.byref(d), int(groups))) > 0


@torch.library.custom_op(f"{LIB}::conv2d_gn_silu", mutates_args=())
def conv2d_gn_silu(x: Tensor, x2: Optional[Tensor], weight: Tensor, bias: Optional[Tensor], pad: int, mode: int,
                   gamma: Tensor, beta: Tensor, scale_shift: Optional[Tensor], groups: int, eps: float,
                   post: Optional[Tensor]) -> Tensor:
    """Block.forward (diffusion.py:142-149): SiLU(GroupNorm(conv(x')) * (scale + 1) + shift) [+ post],
    the GroupNorm statistics accumulated by the conv's epilogue (two launches)."""
    _hip.require_device(x)
    x = x.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    d, shape = _conv_desc(x, x2, weight, pad, mode)
    L = _hip.lib()
    nws = int(L.rdq_conv2d_gn_ws_bytes(ctypes.byref(d), int(groups)))
    if nws == 0:
        raise ValueError("conv2d_gn_silu: shape not supported by the fused form (see conv_gn_fusable)")
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    tk = _tickets(x.device, int(L.rdq_conv2d_tickets(ctypes.byref(d))))
    y = torch.empty(shape, device=x.device, dtype=torch.float32)
    ss = scale_shift.contiguous() if scale_shift is not None else None
    pr = post.contiguous() if post is not None else None
    _hip.check(L.rdq_conv2d_gn_silu(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(weight.contiguous()),
                                    _hip.ptr(bias), int(groups), float(eps), _hip.ptr(gamma), _hip.ptr(beta),
                                    _hip.ptr(ss), _hip.ptr(pr), _hip.ptr(y), _hip.ptr(ws), nws, tk,
                                    _hip.stream_of(x)), "rdq_conv2d_gn_silu")
    return y


@conv2d_gn_silu.register_fake
def _(x, x2, weight, bias, pad, mode, gamma, beta, scale_shift, groups, eps, post):
    _, shape = _conv_desc(x, x2, weight, pad, mode)
    return x.new_empty(shape)


def conv_gn_bf16_fusable(x, x2, weight, pad, mode, groups):
    """rdq_conv2d_bf16_gn_silu applies (the bf16 halo-staged conv, H*W >= 256, C / G in {8, 16, 32, 64})."""
    d, _ = _conv_desc(x, x2, weight, pad, mode)
    return bf16_eligible(weight) and int(_hip.lib().rdq_conv2d_bf16_gn_ws_bytes(ctypes.byref(d), int(groups))) > 0


@torch.library.custom_op(f"{LIB}::conv2d_bf16_gn_silu", mutates_args=())
def conv2d_bf16_gn_silu(x: Tensor, x2: Optional[Tensor], weight: Tensor, bias: Optional[Tensor], pad: int, mode: int,
                        gamma: Tensor, beta: Tensor, scale_shift: Optional[Tensor], groups: int, eps: float,
                        post: Optional[Tensor]) -> Tensor:
    """conv2d_gn_silu with bf16 conv operands (fp32 accumulation): the configs[4] batched U-Net's Block, the
    GroupNorm statistics reduced in the halo-staged conv's epilogue (two launches)."""
    _hip.require_device(x)
    x = x.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    d, shape = _conv_desc(x, x2, weight, pad, mode)
    L = _hip.lib()
    nws = int(L.rdq_conv2d_bf16_gn_ws_bytes(ctypes.byref(d), int(groups)))
    if nws == 0 or not bf16_eligible(weight):
        raise ValueError("conv2d_bf16_gn_silu: shape not supported by the fused form (see conv_gn_bf16_fusable)")
    st = _hip.stream_of(x)
    wp = _bf16_pack(weight, d, st)
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    y = torch.empty(shape, device=x.device, dtype=torch.float32)
    ss = scale_shift.contiguous() if scale_shift is not None else None
    pr = post.contiguous() if post is not None else None
    _hip.check(L.rdq_conv2d_bf16_gn_silu(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(wp), _hip.ptr(bias),
                                         int(groups), float(eps), _hip.ptr(gamma), _hip.ptr(beta), _hip.ptr(ss),
                                         _hip.ptr(pr), _hip.ptr(y), _hip.ptr(ws), nws, st), "rdq_conv2d_bf16_gn_silu")
    return y


@conv2d_bf16_gn_silu.register_fake
def _(x, x2, weight, bias, pad, mode, gamma, beta, scale_shift, groups, eps, post):
    _, shape = _conv_desc(x, x2, weight, pad, mode)
    return x.new_empty(shape)


@torch.library.custom_op(f"{LIB}::conv2d_bf16_block_pair", mutates_args=())
def conv2d_bf16_block_pair(x: Tensor, x2: Optional[Tensor], w1: Tensor, b1: Optional[Tensor], gamma1: Tensor, beta1: Tensor,
                           scale_shift: Optional[Tensor], eps1: float, w2: Tensor, b2: Optional[Tensor], gamma2: Tensor,
                           beta2: Tensor, eps2: float, groups: int, post: Optional[Tensor]) -> Tensor:
    """ResnetBlock's block2(block1(cat(x, x2), scale_shift)) [+ post] on the bf16 halo-staged conv
    (diffusion.py:160-168): block1's normalised output is written as bf16 channel octets, the rounding
    block2's conv applies to its operands anyway (rdq_conv2d_bf16_gn_silu8 / _x8): bit-identical to two
    conv2d_bf16_gn_silu calls, half the bytes between them."""
    _hip.require_device(x)
    x = x.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    d1, shape1 = _conv_desc(x, x2, w1, 1, 0)
    d2, shape2 = _conv_desc(torch.empty(shape1, device="meta"), None, w2, 1, 0)
    L = _hip.lib()
    n1 = int(L.rdq_conv2d_bf16_gn_ws_bytes(ctypes.byref(d1), int(groups)))
    n2 = int(L.rdq_conv2d_bf16_gn_ws_bytes(ctypes.byref(d2), int(groups)))
    if n1 == 0 or n2 == 0 or not bf16_eligible(w1) or not bf16_eligible(w2) or shape1[1] % 32:
        raise ValueError("conv2d_bf16_block_pair: shapes not supported (see unet_ops.block_pair)")
    st = _hip.stream_of(x)
    wp1, wp2 = _bf16_pack(w1, d1, st), _bf16_pack(w2, d2, st)
    ws = torch.empty(max(n1, n2), dtype=torch.uint8, device=x.device)
    B, C1, H, W = shape1
    h8 = torch.empty((B, C1 // 8, H, W, 8), device=x.device, dtype=torch.bfloat16)
    y = torch.empty(shape2, device=x.device, dtype=torch.float32)
    ss = scale_shift.contiguous() if scale_shift is not None else None
    pr = post.contiguous() if post is not None else None
    _hip.check(L.rdq_conv2d_bf16_gn_silu8(ctypes.byref(d1), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(wp1), _hip.ptr(b1),
                                          int(groups), float(eps1), _hip.ptr(gamma1), _hip.ptr(beta1), _hip.ptr(ss),
                                          _hip.ptr(h8), _hip.ptr(ws), n1, st), "rdq_conv2d_bf16_gn_silu8")
    _hip.check(L.rdq_conv2d_bf16_gn_silu_x8(ctypes.byref(d2), _hip.ptr(h8), _hip.ptr(wp2), _hip.ptr(b2), int(groups),
                                            float(eps2), _hip.ptr(gamma2), _hip.ptr(beta2), None, _hip.ptr(pr),
                                            _hip.ptr(y), _hip.ptr(ws), n2, st), "rdq_conv2d_bf16_gn_silu_x8")
    return y


@conv2d_bf16_block_pair.register_fake
def _(x, x2, w1, b1, gamma1, beta1, scale_shift, eps1, w2, b2, gamma2, beta2, eps2, groups, post):
    return x.new_empty((x.shape[0], w2.shape[0], x.shape[2], x.shape[3]))


@torch.library.custom_op(f"{LIB}::conv2d_bf16_gn_silu_out", mutates_args=())
def conv2d_bf16_gn_silu_out(x: Tensor, weight: Tensor, bias: Optional[Tensor], pad: int, gamma: Tensor, beta: Tensor,
                            scale_shift: Optional[Tensor], groups: int, eps: float, post: Optional[Tensor],
                            w_out: Tensor, b_out: Optional[Tensor]) -> Tensor:
    """conv2d_gn_silu_out on the bf16 halo-staged conv (the configs[4] batched U-Net's tail)."""
    _hip.require_device(x)
    x = x.contiguous()
    d, shape = _conv_desc(x, None, weight, pad, 0)
    L = _hip.lib()
    nws = int(L.rdq_conv2d_bf16_gn_ws_bytes(ctypes.byref(d), int(groups)))
    if nws == 0 or not bf16_eligible(weight):
        raise ValueError("conv2d_bf16_gn_silu_out: shape not supported by the fused form (see conv_gn_bf16_fusable)")
    st = _hip.stream_of(x)
    wp = _bf16_pack(weight, d, st)
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    nf = int(w_out.shape[0])
    yf = torch.empty(shape[0], nf, shape[2], shape[3], device=x.device, dtype=torch.float32)
    ss = scale_shift.contiguous() if scale_shift is not None else None
    pr = post.contiguous() if post is not None else None
    _hip.check(L.rdq_conv2d_bf16_gn_silu_out(ctypes.byref(d), _hip.ptr(x), None, _hip.ptr(wp), _hip.ptr(bias),
                                             int(groups), float(eps), _hip.ptr(gamma), _hip.ptr(beta), _hip.ptr(ss),
                                             _hip.ptr(pr), nf, _hip.ptr(w_out.contiguous()), _hip.ptr(b_out),
                                             _hip.ptr(yf), _hip.ptr(ws), nws, st), "rdq_conv2d_bf16_gn_silu_out")
    return yf


@conv2d_bf16_gn_silu_out.register_fake
def _(x, weight, bias, pad, gamma, beta, scale_shift, groups, eps, post, w_out, b_out):
    _, shape = _conv_desc(x, None, weight, pad, 0)
    return x.new_empty(shape[0], w_out.shape[0], shape[2], shape[3])


def conv_gn_sc_fusable(x, x2, weight, weight_s, groups):
    """rdq_conv2d_gn_silu_sc applies: block1's 3x3 conv + GroupNorm (conv_gn_fusable) and a 1x1
    shortcut of the same input in the channel-chunk form (channel counts multiples of 64)."""
    d, _ = _conv_desc(x, x2, weight, 1, 0)
    return weight.shape[-1] == 3 and weight_s.shape[-1] == 1 and \
        int(_hip.lib().rdq_conv2d_gn_sc_ws_bytes(ctypes.byref(d), int(groups), int(weight_s.shape[0]))) > 0


@torch.library.custom_op(f"{LIB}::conv2d_gn_silu_sc", mutates_args=())
def conv2d_gn_silu_sc(x: Tensor, x2: Optional[Tensor], weight: Tensor, bias: Optional[Tensor], gamma: Tensor,
                      beta: Tensor, scale_shift: Optional[Tensor], groups: int, eps: float, weight_s: Tensor,
                      bias_s: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """ResnetBlock with a 1x1 shortcut (diffusion.py:160-168): (block1(cat(x, x2)), res_conv(cat(x, x2)))
    with both convs in one launch, then block1's normalise pass."""
    _hip.require_device(x)
    x = x.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    d, shape = _conv_desc(x, x2, weight, 1, 0)
    cs = int(weight_s.shape[0])
    L = _hip.lib()
    nws = int(L.rdq_conv2d_gn_sc_ws_bytes(ctypes.byref(d), int(groups), cs))
    if nws == 0:
        raise ValueError("conv2d_gn_silu_sc: shape not supported by the fused form (see conv_gn_sc_fusable)")
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    tk = _tickets(x.device, int(L.rdq_conv2d_gn_sc_tickets(ctypes.byref(d), cs)))
    y = torch.empty(shape, device=x.device, dtype=torch.float32)
    ys = torch.empty(shape[0], cs, shape[2], shape[3], device=x.device, dtype=torch.float32)
    ss = scale_shift.contiguous() if scale_shift is not None else None
    _hip.check(L.rdq_conv2d_gn_silu_sc(ctypes.byref(d), _hip.ptr(x), _hip.ptr(x2), _hip.ptr(weight.contiguous()),
                                       _hip.ptr(bias), int(groups), float(eps), _hip.ptr(gamma), _hip.ptr(beta),
                                       _hip.ptr(ss), _hip.ptr(y), cs, _hip.ptr(weight_s.contiguous()), _hip.ptr(bias_s),
                                       _hip.ptr(ys), _hip.ptr(ws), nws, tk, _hip.stream_of(x)),
               "rdq_conv2d_gn_silu_sc")
    return y, ys


@conv2d_gn_silu_sc.register_fake
def _(x, x2, weight, bias, gamma, beta, scale_shift, groups, eps, weight_s, bias_s):
    _, shape = _conv_desc(x, x2, weight, 1, 0)
    return x.new_empty(shape), x.new_empty(shape[0], weight_s.shape[0], shape[2], shape[3])


def _ptr_array(ts):
    return (ctypes.c_void_p * len(ts))(*[_hip.ptr(t) for t in ts])


@torch.library.custom_op(f"{LIB}::conv2d_gn_silu_lsm", mutates_args=())
def conv2d_gn_silu_lsm(x: Tensor, weight: Tensor, bias: Optional[Tensor], pad: int, gamma: Tensor, beta: Tensor,
                       groups: int, eps: float, post: Optional[Tensor], temb: Tensor, weights: List[Tensor],
                       biases: List[Tensor], ss_index: int) -> Tuple[Tensor, List[Tensor]]:
    """(conv2d_gn_silu(x, ..., scale_shift = ys[ss_index], post), ys = linear_silu_multi(temb, weights,
    biases)): the first ResnetBlock's block1 with every block's Linear(SiLU(t)) computed as a side job of
    its conv launch (diffusion.py:280-283, 160-165)."""
    _hip.require_device(x)
    x = x.contiguous()
    temb = temb.contiguous()
    d, shape = _conv_desc(x, None, weight, pad, 0)
    L = _hip.lib()
    nws = int(L.rdq_conv2d_gn_ws_bytes(ctypes.byref(d), int(groups)))
    if nws == 0 or len(weights) > 32:
        raise ValueError("conv2d_gn_silu_lsm: shape not supported by the fused form")
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    tk = _tickets(x.device, int(L.rdq_conv2d_tickets(ctypes.byref(d))))
    y = torch.empty(shape, device=x.device, dtype=torch.float32)
    B, fin = temb.shape
    wl = [w.contiguous() for w in weights]
    ys = [torch.empty(B, w.shape[0], device=x.device, dtype=torch.float32) for w in wl]
    O = (ctypes.c_int32 * len(wl))(*[w.shape[0] for w in wl])
    pr = post.contiguous() if post is not None else None
    _hip.check(L.rdq_conv2d_gn_silu_lsm(ctypes.byref(d), _hip.ptr(x), None, _hip.ptr(weight.contiguous()),
                                        _hip.ptr(bias), int(groups), float(eps), _hip.ptr(gamma), _hip.ptr(beta),
                                        _hip.ptr(pr), _hip.ptr(y), _hip.ptr(ws), nws, tk, fin, _hip.ptr(temb), len(wl),
                                        _ptr_array(wl), _ptr_array(biases), O, _ptr_array(ys), int(ss_index),
                                        _hip.stream_of(x)), "rdq_conv2d_gn_silu_lsm")
    return y, ys


@conv2d_gn_silu_lsm.register_fake
def _(x, weight, bias, pad, gamma, beta, groups, eps, post, temb, weights, biases, ss_index):
    _, shape = _conv_desc(x, None, weight, pad, 0)
    return x.new_empty(shape), [temb.new_empty(temb.shape[0], w.shape[0]) for w in weights]


@torch.library.custom_op(f"{LIB}::conv2d_gn_silu_out", mutates_args=())
def conv2d_gn_silu_out(x: Tensor, weight: Tensor, bias: Optional[Tensor], pad: int, gamma: Tensor, beta: Tensor,
                       scale_shift: Optional[Tensor], groups: int, eps: float, post: Optional[Tensor],
                       w_out: Tensor, b_out: Optional[Tensor]) -> Tensor:
    """conv1x1(conv2d_gn_silu(x, ..., post), w_out) + b_out: final_res_block's block2 and final_conv
    (diffusion.py:299-301), the block output never written (w_out: (nf <= 4, cout, 1, 1))."""
    _hip.require_device(x)
    x = x.contiguous()
    d, shape = _conv_desc(x, None, weight, pad, 0)
    L = _hip.lib()
    nws = int(L.rdq_conv2d_gn_ws_bytes(ctypes.byref(d), int(groups)))
    if nws == 0:
        raise ValueError("conv2d_gn_silu_out: shape not supported by the fused form")
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    tk = _tickets(x.device, int(L.rdq_conv2d_tickets(ctypes.byref(d))))
    nf = int(w_out.shape[0])
    yf = torch.empty(shape[0], nf, shape[2], shape[3], device=x.device, dtype=torch.float32)
    ss = scale_shift.contiguous() if scale_shift is not None else None
    pr = post.contiguous() if post is not None else None
    _hip.check(L.rdq_conv2d_gn_silu_out(ctypes.byref(d), _hip.ptr(x), None, _hip.ptr(weight.contiguous()),
                                        _hip.ptr(bias), int(groups), float(eps), _hip.ptr(gamma), _hip.ptr(beta),
                                        _hip.ptr(ss), _hip.ptr(pr), nf, _hip.ptr(w_out.contiguous()), _hip.ptr(b_out),
                                        _hip.ptr(yf), _hip.ptr(ws), nws, tk, _hip.stream_of(x)),
               "rdq_conv2d_gn_silu_out")
    return yf


@conv2d_gn_silu_out.register_fake
def _(x, weight, bias, pad, gamma, beta, scale_shift, groups, eps, post, w_out, b_out):
    _, shape = _conv_desc(x, None, weight, pad, 0)
    return x.new_empty(shape[0], w_out.shape[0], shape[2], shape[3])


def unet_head_fusable(x, weight, time_mlp):
    """rdq_unet_head applies: init_conv outside the channel-chunk form (7x7 / 3x3, cout <= 64, no K split), B <= 16
    (beyond, the time MLP's batched kernel reads its weights once per sample block instead)."""
    cout, cin, kh, kw = weight.shape
    dim, hid = time_mlp[1].weight.shape[1], time_mlp[1].weight.shape[0]
    return x.shape[0] <= 16 and kh == kw and kh in (3, 7) and cout <= 64 and cin * kh * kw <= 224 and \
        x.shape[1] == cin and \
        (kh == 7 or cin % 8 != 0) and dim + hid <= 7680


@torch.library.custom_op(f"{LIB}::unet_head", mutates_args=())
def unet_head(x: Tensor, weight: Tensor, bias: Optional[Tensor], pad: int, t: Tensor, dim: int, theta: float,
              w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor) -> Tuple[Tensor, Tensor]:
    """(init_conv(x), time_mlp(t)) in one launch (diffusion.py:276-279)."""
    _hip.require_device(x)
    x = x.contiguous()
    t = t.to(torch.int64).contiguous()
    d, shape = _conv_desc(x, None, weight, pad, 0)
    y = torch.empty(shape, device=x.device, dtype=torch.float32)
    hid, out = w1.shape[0], w2.shape[0]
    temb = torch.empty(t.shape[0], out, device=x.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_unet_head(ctypes.byref(d), _hip.ptr(x), _hip.ptr(weight.contiguous()), _hip.ptr(bias),
                                        _hip.ptr(y), dim, float(theta), _hip.ptr(t), _hip.ptr(w1.contiguous()),
                                        _hip.ptr(b1), hid, _hip.ptr(w2.contiguous()), _hip.ptr(b2), out,
                                        _hip.ptr(temb), _hip.stream_of(x)), "rdq_unet_head")
    return y, temb


@unet_head.register_fake
def _(x, weight, bias, pad, t, dim, theta, w1, b1, w2, b2):
    _, shape = _conv_desc(x, None, weight, pad, 0)
    return x.new_empty(shape), x.new_empty(t.shape[0], w2.shape[0])


@torch.library.custom_op(f"{LIB}::rmsnorm", mutates_args=())
def rmsnorm(x: Tensor, g: Tensor, residual: Optional[Tensor]) -> Tensor:
    """F.normalize(x, dim=1) * g * sqrt(C) [+ residual]."""
    _hip.require_device(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    y = torch.empty_like(x)
    res = residual.contiguous() if residual is not None else None
    _hip.check(_hip.lib().rdq_rmsnorm(B, C, H * W, _hip.ptr(x), _hip.ptr(g), _hip.ptr(res), _hip.ptr(y),
                                      _hip.stream_of(x)), "rdq_rmsnorm")
    return y


@rmsnorm.register_fake
def _(x, g, residual):
    return torch.empty_like(x)


@torch.library.custom_op(f"{LIB}::linear", mutates_args=())
def linear(x: Tensor, weight: Tensor, bias: Tensor, act_in: int, act_out: int) -> Tensor:
    """act_out(Linear(act_in(x))); act 1 = SiLU on the input / GELU(erf) on the output."""
    _hip.require_device(x)
    x = x.contiguous()
    B, fin = x.shape
    fout = weight.shape[0]
    y = torch.empty(B, fout, device=x.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_linear(B, fin, fout, _hip.ptr(x), _hip.ptr(weight), _hip.ptr(bias), act_in, act_out,
                                     _hip.ptr(y), _hip.stream_of(x)), "rdq_linear")
    return y


@linear.register_fake
def _(x, weight, bias, act_in, act_out):
    return x.new_empty(x.shape[0], weight.shape[0])


@torch.library.custom_op(f"{LIB}::time_mlp", mutates_args=())
def time_mlp(t: Tensor, dim: int, theta: float, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor) -> Tensor:
    """Unet.time_mlp (diffusion.py:255-258): Linear(GELU(Linear(SinusoidalPosEmb(t)))), one launch."""
    _hip.require_device(t)
    t = t.to(torch.int64).contiguous()
    hid, out = w1.shape[0], w2.shape[0]
    y = torch.empty(t.shape[0], out, device=t.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_time_mlp(t.shape[0], dim, float(theta), _hip.ptr(t), _hip.ptr(w1.contiguous()),
                                       _hip.ptr(b1), hid, _hip.ptr(w2.contiguous()), _hip.ptr(b2), out, _hip.ptr(y),
                                       _hip.stream_of(t)), "rdq_time_mlp")
    return y


@time_mlp.register_fake
def _(t, dim, theta, w1, b1, w2, b2):
    return t.new_empty(t.shape[0], w2.shape[0], dtype=torch.float32)


@torch.library.custom_op(f"{LIB}::linear_silu_multi", mutates_args=())
def linear_silu_multi(x: Tensor, weights: List[Tensor], biases: List[Tensor]) -> List[Tensor]:
    """[Linear_j(SiLU(x)) for j]: every ResnetBlock's time MLP (diffusion.py:157-165), one launch
    (at most 32 linears sharing x)."""
    _hip.require_device(x)
    x = x.contiguous()
    n = len(weights)
    B, fin = x.shape
    ys = [torch.empty(B, w.shape[0], device=x.device, dtype=torch.float32) for w in weights]
    ws = [w.contiguous() for w in weights]
    W = (ctypes.c_void_p * n)(*[_hip.ptr(w) for w in ws])
    Bs = (ctypes.c_void_p * n)(*[_hip.ptr(b) for b in biases])
    O = (ctypes.c_int32 * n)(*[w.shape[0] for w in ws])
    Y = (ctypes.c_void_p * n)(*[_hip.ptr(y) for y in ys])
    _hip.check(_hip.lib().rdq_linear_silu_multi(B, fin, _hip.ptr(x), n, W, Bs, O, Y, _hip.stream_of(x)),
               "rdq_linear_silu_multi")
    return ys


@linear_silu_multi.register_fake
def _(x, weights, biases):
    return [x.new_empty(x.shape[0], w.shape[0]) for w in weights]


@torch.library.custom_op(f"{LIB}::sinusoidal_emb", mutates_args=())
def sinusoidal_emb(t: Tensor, dim: int, theta: float) -> Tensor:
    _hip.require_device(t)
    t = t.to(torch.int64).contiguous()
    y = torch.empty(t.shape[0], dim, device=t.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_sinusoidal_emb(t.shape[0], dim, float(theta), _hip.ptr(t), _hip.ptr(y),
                                             _hip.stream_of(t)), "rdq_sinusoidal_emb")
    return y


@sinusoidal_emb.register_fake
def _(t, dim, theta):
    return t.new_empty(t.shape[0], dim, dtype=torch.float32)


@torch.library.custom_op(f"{LIB}::linear_attn", mutates_args=())
def linear_attn(qkv: Tensor, mem_kv: Tensor, heads: int, scale: float) -> Tensor:
    """LinearAttention core (diffusion.py:182-195): softmax(q) over d, softmax(k) over n with the
    memory key/values, context, out = context^T q; qkv (B, 3*heads*dh, H, W) -> (B, heads*dh, H, W)."""
    _hip.require_device(qkv)
    qkv = qkv.contiguous()
    B, C3, H, W = qkv.shape
    dh = C3 // (3 * heads)
    L = _hip.lib()
    ws = torch.empty(int(L.rdq_linear_attention_ws_bytes(B, heads, dh, H * W, mem_kv.shape[-1])), dtype=torch.uint8,
                     device=qkv.device)
    out = torch.empty(B, heads * dh, H, W, device=qkv.device, dtype=torch.float32)
    _hip.check(L.rdq_linear_attention(B, heads, dh, H * W, mem_kv.shape[-1], float(scale), _hip.ptr(qkv),
                                      _hip.ptr(mem_kv.contiguous()), _hip.ptr(out), _hip.ptr(ws), _hip.stream_of(qkv)),
               "rdq_linear_attention")
    return out


@linear_attn.register_fake
def _(qkv, mem_kv, heads, scale):
    B, C3, H, W = qkv.shape
    return qkv.new_empty(B, C3 // 3, H, W)


def linear_attn_block_fusable(qkv_channels, heads, dim):
    return heads == 4 and qkv_channels == 3 * heads * 32 and dim in (64, 128, 256)


@torch.library.custom_op(f"{LIB}::linear_attn_block", mutates_args=())
def linear_attn_block(qkv: Tensor, mem_kv: Tensor, heads: int, scale: float, w_out: Tensor,
                      b_out: Optional[Tensor], g_out: Tensor, residual: Optional[Tensor]) -> Tensor:
    """LinearAttention.forward(x) + x from qkv = to_qkv(RMSNorm(x)) (diffusion.py:182-195, residual
    286/297): context, softmax(q) x context, to_out = Conv2d(hidden, dim, 1) + RMSNorm(dim) and the
    residual, the last four in one launch (rdq_linear_attention_block).  dh = 32, dim 64/128/256."""
    _hip.require_device(qkv)
    qkv = qkv.contiguous()
    B, C3, H, W = qkv.shape
    dh = C3 // (3 * heads)
    dim = w_out.shape[0]
    L = _hip.lib()
    ws = torch.empty(int(L.rdq_linear_attention_ws_bytes(B, heads, dh, H * W, mem_kv.shape[-1])), dtype=torch.uint8,
                     device=qkv.device)
    y = torch.empty(B, dim, H, W, device=qkv.device, dtype=torch.float32)
    res = residual.contiguous() if residual is not None else None
    _hip.check(L.rdq_linear_attention_block(B, heads, dh, H * W, mem_kv.shape[-1], float(scale), _hip.ptr(qkv),
                                            _hip.ptr(mem_kv.contiguous()), dim, _hip.ptr(w_out.contiguous()),
                                            _hip.ptr(b_out) if b_out is not None else None,
                                            _hip.ptr(g_out.contiguous()), _hip.ptr(res) if res is not None else None,
                                            _hip.ptr(y), _hip.ptr(ws), _hip.stream_of(qkv)),
               "rdq_linear_attention_block")
    return y


@linear_attn_block.register_fake
def _(qkv, mem_kv, heads, scale, w_out, b_out, g_out, residual):
    B, C3, H, W = qkv.shape
    return qkv.new_empty(B, w_out.shape[0], H, W)


def linear_attn_bf16_fusable(x, w_qkv, w_out, heads):
    """rdq_linear_attention_bf16 applies: 4 heads of 32, dim 64 / 128 (the U-Net's 72 / 36 / 18 levels), 1x1 projections."""
    return (heads == 4 and x.dim() == 4 and x.shape[1] in (64, 128) and tuple(w_qkv.shape) == (384, x.shape[1], 1, 1)
            and tuple(w_out.shape) == (x.shape[1], 128, 1, 1))


@torch.library.custom_op(f"{LIB}::linear_attn_bf16", mutates_args=())
def linear_attn_bf16(x: Tensor, g_in: Tensor, w_qkv: Tensor, mem_kv: Tensor, w_out: Tensor, b_out: Optional[Tensor],
                     g_out: Tensor, heads: int, scale: float) -> Tensor:
    """LinearAttention.forward(x) + x (diffusion.py:182-195, residual 286/297) with bf16 operands and fp32
    accumulation, two launches (rdq_linear_attention_bf16): the configs[4] batched U-Net."""
    _hip.require_device(x)
    if not linear_attn_bf16_fusable(x, w_qkv, w_out, heads):
        raise ValueError("linear_attn_bf16: shape not supported (see linear_attn_bf16_fusable)")
    x = x.contiguous()
    B, D, H, W = x.shape
    L = _hip.lib()
    st = _hip.stream_of(x)
    dq, _ = _conv_desc(x, None, w_qkv, 0, 0)
    h = torch.empty(B, 128, H, W, device="meta")
    do, _ = _conv_desc(h, None, w_out, 0, 0)
    wq = _bf16_pack(w_qkv, dq, st)
    wo = _bf16_pack(w_out, do, st)
    nws = int(L.rdq_linear_attention_bf16_ws_bytes(B, D, H * W))
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    y = torch.empty_like(x)
    _hip.check(L.rdq_linear_attention_bf16(B, D, H * W, mem_kv.shape[-1], float(scale), _hip.ptr(x),
                                           _hip.ptr(g_in.contiguous()), _hip.ptr(wq), _hip.ptr(mem_kv.contiguous()),
                                           _hip.ptr(wo), _hip.ptr(b_out) if b_out is not None else None,
                                           _hip.ptr(g_out.contiguous()), _hip.ptr(y), _hip.ptr(ws), nws, st),
               "rdq_linear_attention_bf16")
    return y


@linear_attn_bf16.register_fake
def _(x, g_in, w_qkv, mem_kv, w_out, b_out, g_out, heads, scale):
    return torch.empty_like(x)


@torch.library.custom_op(f"{LIB}::linear_attn_f32", mutates_args=())
def linear_attn_f32(x: Tensor, g_in: Tensor, w_qkv: Tensor, mem_kv: Tensor, w_out: Tensor, b_out: Optional[Tensor],
                    g_out: Tensor, heads: int, scale: float) -> Tensor:
    """LinearAttention.forward(x) + x (diffusion.py:182-195, residual 286/297) in fp32, two launches
    (rdq_linear_attention_f32: qkv and the hidden tensor never written)."""
    _hip.require_device(x)
    if not linear_attn_bf16_fusable(x, w_qkv, w_out, heads):
        raise ValueError("linear_attn_f32: shape not supported (see linear_attn_bf16_fusable)")
    x = x.contiguous()
    B, D, H, W = x.shape
    L = _hip.lib()
    nws = int(L.rdq_linear_attention_f32_ws_bytes(B, D, H * W))
    ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
    y = torch.empty_like(x)
    _hip.check(L.rdq_linear_attention_f32(B, D, H * W, mem_kv.shape[-1], float(scale), _hip.ptr(x),
                                          _hip.ptr(g_in.contiguous()), _hip.ptr(w_qkv.contiguous()),
                                          _hip.ptr(mem_kv.contiguous()), _hip.ptr(w_out.contiguous()),
                                          _hip.ptr(b_out) if b_out is not None else None, _hip.ptr(g_out.contiguous()),
                                          _hip.ptr(y), _hip.ptr(ws), nws, _hip.stream_of(x)), "rdq_linear_attention_f32")
    return y


@linear_attn_f32.register_fake
def _(x, g_in, w_qkv, mem_kv, w_out, b_out, g_out, heads, scale):
    return torch.empty_like(x)


@torch.library.custom_op(f"{LIB}::attn", mutates_args=())
def attn(qkv: Tensor, mem_kv: Tensor, heads: int) -> Tensor:
    """Attention core with Attend(flash=False) (diffusion.py:209-218): softmax(q k^T d^-1/2) v over
    the memory + image keys; qkv (B, 3*heads*dh, H, W) -> (B, heads*dh, H, W)."""
    _hip.require_device(qkv)
    qkv = qkv.contiguous()
    B, C3, H, W = qkv.shape
    dh = C3 // (3 * heads)
    out = torch.empty(B, heads * dh, H, W, device=qkv.device, dtype=torch.float32)
    _hip.check(_hip.lib().rdq_full_attention(B, heads, dh, H * W, mem_kv.shape[-2], _hip.ptr(qkv),
                                             _hip.ptr(mem_kv.contiguous()), _hip.ptr(out), _hip.stream_of(qkv)),
               "rdq_full_attention")
    return out


@attn.register_fake
def _(qkv, mem_kv, heads):
    B, C3, H, W = qkv.shape
    return qkv.new_empty(B, C3 // 3, H, W)


@torch.library.custom_op(f"{LIB}::red_q_sample", mutates_args=())
def red_q_sample(x0: Tensor, t: Tensor, eps: Tensor, sqrt_ac: Tensor, sqrt_1mac: Tensor) -> Tensor:
    """q_sample (diffusion.py:516-519) on the fp32 schedule buffers."""
    _hip.require_device(x0)
    x0, eps = x0.contiguous(), eps.contiguous()
    xt = torch.empty_like(x0)
    _hip.check(_hip.lib().rdq_red_q_sample(x0.shape[0], x0[0].numel(), _hip.ptr(sqrt_ac), _hip.ptr(sqrt_1mac),
                                           _hip.ptr(t), _hip.ptr(x0), _hip.ptr(eps), _hip.ptr(xt),
                                           _hip.stream_of(x0)), "rdq_red_q_sample")
    return xt


@torch.library.custom_op(f"{LIB}::red_q_sample_into", mutates_args=("xt", "t_out"))
def red_q_sample_into(x0: Tensor, t: Tensor, eps: Tensor, sqrt_ac: Tensor, sqrt_1mac: Tensor, xt: Tensor,
                      t_out: Tensor) -> None:
    """red_q_sample written into xt (contiguous, x0's shape), t copied into t_out (int64 [B]) by the same
    launch: the static inputs of a captured U-Net forward (Unet.graph_io)."""
    _hip.require_device(x0)
    x0, eps = x0.contiguous(), eps.contiguous()
    if xt.shape != x0.shape or not xt.is_contiguous() or t_out.dtype != torch.int64 or t_out.numel() != x0.shape[0]:
        raise ValueError("red_q_sample_into: xt / t_out do not match x0")
    _hip.check(_hip.lib().rdq_red_q_sample_t(x0.shape[0], x0[0].numel(), _hip.ptr(sqrt_ac), _hip.ptr(sqrt_1mac),
                                             _hip.ptr(t.to(torch.int64).contiguous()), _hip.ptr(x0), _hip.ptr(eps),
                                             _hip.ptr(xt), _hip.ptr(t_out), _hip.stream_of(x0)), "rdq_red_q_sample_t")


@red_q_sample_into.register_fake
def _(x0, t, eps, sqrt_ac, sqrt_1mac, xt, t_out):
    return None


@red_q_sample.register_fake
def _(x0, t, eps, sqrt_ac, sqrt_1mac):
    return torch.empty_like(x0)


@torch.library.custom_op(f"{LIB}::red_eps", mutates_args=())
def red_eps(xt: Tensor, t: Tensor, eps_hat: Tensor, eps: Tensor, sqrt_recip_ac: Tensor,
            sqrt_recipm1_ac: Tensor) -> Tensor:
    """RED residual (eps' - eps): eps' re-derived from the clipped x0 (diffusion.py:393-419)."""
    _hip.require_device(xt)
    xt, eps_hat, eps = xt.contiguous(), eps_hat.contiguous(), eps.contiguous()
    g = torch.empty_like(xt)
    _hip.check(_hip.lib().rdq_red_epilogue(xt.shape[0], xt[0].numel(), _hip.ptr(sqrt_recip_ac),
                                           _hip.ptr(sqrt_recipm1_ac), _hip.ptr(t), _hip.ptr(xt), _hip.ptr(eps_hat),
                                           _hip.ptr(eps), _hip.ptr(g), _hip.stream_of(xt)), "rdq_red_epilogue")
    return g


@red_eps.register_fake
def _(xt, t, eps_hat, eps, sqrt_recip_ac, sqrt_recipm1_ac):
    return torch.empty_like(xt)


# ----------------------------------------------------------------------------------------- loop
@torch.library.custom_op(f"{LIB}::l1_misfit", mutates_args=())
def l1_misfit(pred: Tensor, y: Tensor, mask: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """K5: per-model sum(|y - pred| * mask) / max(#observed, 1) (losses.py:14-41) -> (loss, nobs)."""
    _hip.require_device(pred, y, mask)
    pred, y = pred.float().contiguous(), y.float().contiguous()
    mask = mask.float().contiguous() if mask is not None else None
    B = pred.shape[0]
    n = pred.numel() // B
    L = _hip.lib()
    loss = torch.empty(B, dtype=torch.float32, device=pred.device)
    nobs = torch.empty(B, dtype=torch.float32, device=pred.device)
    part = torch.empty(int(L.rdq_l1_partial_bytes(B, n)), dtype=torch.uint8, device=pred.device)
    _hip.check(L.rdq_l1_forward(B, n, _hip.ptr(pred), _hip.ptr(y), _hip.ptr(mask), _hip.ptr(loss), _hip.ptr(nobs),
                                _hip.ptr(part), _hip.stream_of(pred)), "rdq_l1_forward")
    return loss, nobs


@l1_misfit.register_fake
def _(pred, y, mask):
    return pred.new_empty(pred.shape[0]), pred.new_empty(pred.shape[0])


@torch.library.custom_op(f"{LIB}::l1_misfit_backward", mutates_args=())
def l1_misfit_backward(pred: Tensor, y: Tensor, mask: Optional[Tensor], nobs: Tensor, gout: Tensor) -> Tensor:
    """dL/dpred = sign(pred - y) * mask * gout / nobs (the autograd of losses.py:27-39)."""
    _hip.require_device(pred, y)
    pred, y = pred.float().contiguous(), y.float().contiguous()
    mask = mask.float().contiguous() if mask is not None else None
    B = pred.shape[0]
    dpred = torch.empty_like(pred)
    _hip.check(_hip.lib().rdq_l1_backward(B, pred.numel() // B, _hip.ptr(pred), _hip.ptr(y), _hip.ptr(mask),
                                          _hip.ptr(nobs.float().contiguous()), _hip.ptr(gout.float().contiguous()),
                                          _hip.ptr(dpred), _hip.stream_of(pred)), "rdq_l1_backward")
    return dpred


@l1_misfit_backward.register_fake
def _(pred, y, mask, nobs, gout):
    return torch.empty_like(pred, dtype=torch.float32)


@torch.library.custom_op(f"{LIB}::smooth_reg", mutates_args=())
def smooth_reg(mu: Tensor, kind: int) -> Tensor:
    """K6: TV (kind 0) / Tikhonov (kind 1) per model on the padded model (benchmark.py:4-37)."""
    _hip.require_device(mu)
    m = mu.float().contiguous()
    B, _, H, W = m.shape
    loss = torch.empty(B, dtype=torch.float32, device=m.device)
    _hip.check(_hip.lib().rdq_smooth_reg_forward(kind, B, H, W, _hip.ptr(m), _hip.ptr(loss), _hip.stream_of(m)),
               "rdq_smooth_reg_forward")
    return loss


@smooth_reg.register_fake
def _(mu, kind):
    return mu.new_empty(mu.shape[0], dtype=torch.float32)


@torch.library.custom_op(f"{LIB}::smooth_reg_backward", mutates_args=())
def smooth_reg_backward(mu: Tensor, gout: Tensor, kind: int) -> Tensor:
    _hip.require_device(mu)
    m = mu.float().contiguous()
    B, _, H, W = m.shape
    grad = torch.empty_like(m)
    _hip.check(_hip.lib().rdq_smooth_reg_backward(kind, B, H, W, _hip.ptr(m), _hip.ptr(gout.float().contiguous()),
                                                  _hip.ptr(grad), _hip.stream_of(m)), "rdq_smooth_reg_backward")
    return grad


@smooth_reg_backward.register_fake
def _(mu, gout, kind):
    return torch.empty_like(mu, dtype=torch.float32)


@torch.library.custom_op(f"{LIB}::metrics", mutates_args=())
def metrics(pred: Tensor, true_norm: Tensor) -> Tensor:
    """K12: (mae, rmse, ssim) per model as a (3, B) device tensor (metrics.py:13-46)."""
    _hip.require_device(pred)
    B, _, H, W = pred.shape
    t = true_norm.contiguous()
    L = _hip.lib()
    ws = torch.empty(int(L.rdq_metrics_ws_bytes(B, H, W)), dtype=torch.uint8, device=pred.device)
    out = torch.empty(3, B, dtype=torch.float32, device=pred.device)
    strides = (ctypes.c_int64 * 4)(*pred.stride())
    _hip.check(L.rdq_metrics(B, H, W, _hip.ptr(pred), strides, _hip.ptr(t), _hip.ptr(out), _hip.ptr(ws),
                             _hip.stream_of(pred)), "rdq_metrics")
    return out


@metrics.register_fake
def _(pred, true_norm):
    return pred.new_empty(3, pred.shape[0], dtype=torch.float32)


@torch.library.custom_op(f"{LIB}::adam_clamp_", mutates_args=("param", "exp_avg", "exp_avg_sq"))
def adam_clamp_(param: Tensor, grad: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, beta1: float, beta2: float,
                eps: float, step_size: float, bias_correction2_sqrt: float, clamp: bool, lo: float, hi: float,
                guard: Optional[Tensor] = None) -> None:
    """K11: one torch.optim.Adam step (step_size = -lr / (1 - beta1^t), bias_correction2_sqrt =
    sqrt(1 - beta2^t); torch/optim/adam.py's multi-tensor formula) then param.clamp_(lo, hi) when
    `clamp`, in one launch (reference inversion.py:87-91).  guard: optional int32 device word; the
    step is a no-op on the device while it is non-zero (the FWI status word of a failed persistent
    launch)."""
    _hip.require_device(param)
    for t in (grad, exp_avg, exp_avg_sq):
        if t.shape != param.shape or not t.is_contiguous() or t.dtype != torch.float32:
            raise ValueError("adam_clamp_: grad / exp_avg / exp_avg_sq must be contiguous fp32 like param")
    if not param.is_contiguous() or param.dtype != torch.float32:
        raise ValueError("adam_clamp_: param must be contiguous fp32")
    if guard is not None and (guard.dtype != torch.int32 or guard.numel() < 1):
        raise ValueError("adam_clamp_: guard must be an int32 device word")
    _hip.check(_hip.lib().rdq_adam_step(param.numel(), _hip.ptr(param), _hip.ptr(grad), _hip.ptr(exp_avg),
                                        _hip.ptr(exp_avg_sq), beta1, beta2, eps, step_size, bias_correction2_sqrt,
                                        int(clamp), lo, hi, _hip.ptr(guard), _hip.stream_of(param)),
               "rdq_adam_step")


@adam_clamp_.register_fake
def _(param, grad, exp_avg, exp_avg_sq, beta1, beta2, eps, step_size, bias_correction2_sqrt, clamp, lo, hi,
      guard=None):
    return None


# ------------------------------------------------------------------ forward-only operators
def _forward_only(op, name):
    """The U-Net / regulariser operators are inference kernels (the RED gradient is
    (eps_hat - eps).detach(), regularization/diffusion.py:75): they run with grad-requiring inputs
    (module parameters) but have no backward; differentiating through one raises."""
    def backward(ctx, *grads):
        raise RuntimeError(f"red_diffeq::{name} has no backward (forward-only HIP kernel)")

    def setup(ctx, inputs, output):
        pass
    op.register_autograd(backward, setup_context=setup)


for _op, _name in ((conv2d_mfma, "conv2d_mfma"), (conv2d_rms, "conv2d_rms"), (conv2d_gn_silu, "conv2d_gn_silu"), (conv2d_gn_silu_sc, "conv2d_gn_silu_sc"),
                   (conv2d_bf16_gn_silu, "conv2d_bf16_gn_silu"), (conv2d_bf16_gn_silu_out, "conv2d_bf16_gn_silu_out"),
                   (conv2d_bf16_block_pair, "conv2d_bf16_block_pair"),
                   (conv2d_gn_silu_lsm, "conv2d_gn_silu_lsm"), (conv2d_gn_silu_out, "conv2d_gn_silu_out"), (unet_head, "unet_head"),
                   (gn_silu, "gn_silu"),
                   (rmsnorm, "rmsnorm"), (linear, "linear"), (time_mlp, "time_mlp"),
                   (linear_silu_multi, "linear_silu_multi"),
                   (sinusoidal_emb, "sinusoidal_emb"), (linear_attn, "linear_attn"), (linear_attn_block, "linear_attn_block"), (linear_attn_bf16, "linear_attn_bf16"), (linear_attn_f32, "linear_attn_f32"), (attn, "attn"),
                   (red_q_sample, "red_q_sample"), (red_eps, "red_eps"), (metrics, "metrics")):
    _forward_only(_op, _name)
