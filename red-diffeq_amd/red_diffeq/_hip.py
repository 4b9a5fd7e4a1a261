"""ctypes binding of the in-tree HIP library (C ABI: include/red_diffeq_fwi.h).

The product path has exactly one implementation: the HIP kernels in
red-diffeq_amd/lib/libred_diffeq_hip.so running on an MI355X.  There is no CPU fallback: if the
library is missing, or a tensor is not on a ROCm device, calls raise ``RuntimeError``.
"""
import ctypes
import os

import torch

_PKG = os.path.dirname(os.path.abspath(__file__))
# RDQ_HIP_LIB: another build of the same library (A/B timing of kernel variants, tools/)
LIB_PATH = os.environ.get("RDQ_HIP_LIB") or os.path.join(os.path.dirname(_PKG), "lib", "libred_diffeq_hip.so")

c_int32, c_int64, c_float, c_double, c_size_t, c_void_p = (
    ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p)


class FwiGeom(ctypes.Structure):
    """struct rdq_fwi_geom."""
    _fields_ = [("nz", c_int32), ("nx", c_int32), ("nbc", c_int32), ("nt", c_int32),
                ("ns", c_int32), ("ng", c_int32), ("sample_temporal", c_int32),
                ("dx", c_float), ("dt", c_float), ("isz", c_int32), ("igz", c_int32),
                ("isx", ctypes.POINTER(c_int32)), ("igx", ctypes.POINTER(c_int32)),
                ("wavelet", ctypes.POINTER(c_double))]


class FwiSizes(ctypes.Structure):
    """struct rdq_fwi_sizes_t."""
    _fields_ = [("Hp", c_int32), ("Wp", c_int32), ("ld", c_int32), ("nrec", c_int32),
                ("coeffs", c_size_t), ("vstat", c_size_t), ("seis", c_size_t), ("history", c_size_t),
                ("ring", c_size_t), ("gA", c_size_t), ("gk_part", c_size_t), ("gbeta", c_size_t),
                ("colsum", c_size_t)]


class ConvDesc(ctypes.Structure):
    """struct rdq_conv_desc."""
    _fields_ = [(n, c_int32) for n in ("B", "cin1", "cin2", "H", "W", "cout", "kh", "kw", "pad", "in_mode")]


# name -> (restype, argtypes); must match include/*.h (tests check every symbol)
SIGNATURES = {
    "rdq_fwi_plan_create": (c_int32, [ctypes.POINTER(FwiGeom), ctypes.POINTER(c_void_p)]),
    "rdq_fwi_plan_destroy": (c_int32, [c_void_p]),
    "rdq_fwi_sizes": (c_int32, [c_void_p, c_int32, ctypes.POINTER(FwiSizes)]),
    "rdq_fwi_set_graphs": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_set_tuning": (c_int32, [c_void_p, c_int32, c_int32, c_int32]),
    "rdq_fwi_set_variant": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_set_wide_adj_steps": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_set_wide_adj_shots": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_set_wide_fwd_shots": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_set_wide_fwd_steps": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_set_persistent": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_set_rows_per_wave": (c_int32, [c_void_p, c_int32, c_int32]),
    "rdq_fwi_status": (c_int32, [c_void_p, c_void_p]),
    "rdq_fwi_debug_words": (c_int32, [c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "rdq_fwi_set_status_buffer": (c_int32, [c_void_p, c_void_p]),
    "rdq_fwi_set_profile": (c_int32, [c_void_p, c_int32]),
    "rdq_fwi_profile_waves": (c_int32, [c_void_p, c_int32, ctypes.POINTER(ctypes.c_uint64), c_size_t]),
    "rdq_fwi_launch_info": (c_int32, [c_void_p, c_int32, ctypes.POINTER(c_int32)]),
    "rdq_fwi_wide_info": (c_int32, [c_void_p, c_int32, ctypes.POINTER(c_int32)]),
    "rdq_fwi_set_sweep_delay": (c_int32, [c_void_p, c_int32, c_int32]),
    "rdq_fwi_read_profile": (c_int32, [c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "rdq_fwi_coeffs": (c_int32, [c_void_p, c_int32, c_void_p, ctypes.POINTER(c_int64), c_int32,
                                 c_void_p, c_void_p, c_void_p]),
    "rdq_fwi_forward": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rdq_fwi_adjoint": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p]),
    "rdq_fwi_grad_finalize": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "rdq_l1_partial_bytes": (c_size_t, [c_int32, c_int64]),
    "rdq_l1_forward": (c_int32, [c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p]),
    "rdq_l1_backward": (c_int32, [c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p]),
    "rdq_smooth_reg_forward": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "rdq_smooth_reg_backward": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                          c_void_p, c_void_p]),
    # include/red_diffeq_unet.h
    "rdq_conv2d_ws_bytes": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rdq_conv2d_tickets": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rdq_conv2d": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_size_t, c_void_p, c_void_p]),
    "rdq_conv2d_rms": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_size_t, c_void_p, c_void_p]),
    "rdq_conv2d_gn_ws_bytes": (c_size_t, [ctypes.POINTER(ConvDesc), c_int32]),
    "rdq_conv2d_gn_sc_ws_bytes": (c_size_t, [ctypes.POINTER(ConvDesc), c_int32, c_int32]),
    "rdq_conv2d_gn_sc_tickets": (c_size_t, [ctypes.POINTER(ConvDesc), c_int32]),
    "rdq_conv2d_gn_silu_sc": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                        c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "rdq_conv2d_gn_silu": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                     c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                     c_void_p, c_void_p]),
    "rdq_conv2d_gn_silu_lsm": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                         c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                         c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_int32, c_void_p]),
    "rdq_conv2d_gn_silu_out": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                         c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "rdq_unet_head": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_float,
                                c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "rdq_conv2d_bf16_wpack_bytes": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rdq_conv2d_stem": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rdq_conv2d_bf16_pack": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p]),
    "rdq_conv2d_bf16_ws_bytes": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rdq_unet_set_option": (c_int32, [c_int32, c_int32]),
    "rdq_unet_options_generation": (c_int32, []),
    "rdq_conv2d_bf16": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_size_t, c_void_p]),
    "rdq_conv2d_bf16_gn_ws_bytes": (c_size_t, [ctypes.POINTER(ConvDesc), c_int32]),
    "rdq_conv2d_bf16_gn_silu": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                          c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_size_t, c_void_p]),
    "rdq_conv2d_bf16_gn_silu8": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                           c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                           c_void_p]),
    "rdq_conv2d_bf16_gn_silu_x8": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_int32, c_float,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                             c_void_p]),
    "rdq_conv2d_bf16_gn_silu_out": (c_int32, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_int32, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "rdq_group_norm_ws_bytes": (c_size_t, [c_int32, c_int32, c_int32, c_int32]),
    "rdq_group_norm_silu": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_float, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p]),
    "rdq_rmsnorm": (c_int32, [c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rdq_linear": (c_int32, [c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                             c_void_p]),
    "rdq_time_mlp": (c_int32, [c_int32, c_int32, c_float, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                               c_int32, c_void_p, c_void_p]),
    "rdq_linear_silu_multi": (c_int32, [c_int32, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "rdq_sinusoidal_emb": (c_int32, [c_int32, c_int32, c_float, c_void_p, c_void_p, c_void_p]),
    "rdq_linear_attention_ws_bytes": (c_size_t, [c_int32, c_int32, c_int32, c_int32, c_int32]),
    "rdq_linear_attention": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32, c_float, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    "rdq_linear_attention_block": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32, c_float, c_void_p,
                                             c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p]),
    "rdq_linear_attention_bf16_ws_bytes": (c_size_t, [c_int32, c_int32, c_int32]),
    "rdq_linear_attention_f32_ws_bytes": (c_size_t, [c_int32, c_int32, c_int32]),
    "rdq_linear_attention_f32": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_float, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                           c_void_p]),
    "rdq_linear_attention_bf16": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_float, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                            c_void_p]),
    "rdq_full_attention": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    "rdq_red_q_sample": (c_int32, [c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "rdq_red_q_sample_t": (c_int32, [c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    "rdq_red_epilogue": (c_int32, [c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    # include/red_diffeq_loop.h
    "rdq_adam_step": (c_int32, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_float, c_float,
                                c_float, c_int32, c_float, c_float, c_void_p, c_void_p]),
    "rdq_metrics_ws_bytes": (c_size_t, [c_int32, c_int32, c_int32]),
    "rdq_metrics": (c_int32, [c_int32, c_int32, c_int32, c_void_p, ctypes.POINTER(c_int64), c_void_p, c_void_p, c_void_p,
                              c_void_p]),
}


_lib = None


def load_library():
    """Load the HIP library and declare every exported signature (raises if absent)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"red-diffeq_amd HIP library not built: {LIB_PATH} is missing "
                "(run `make -C red-diffeq_amd` or __graft_entry__.build()).")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


def lib():
    return load_library()


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def require_device(*tensors):
    """The product path runs on a ROCm device only: refuse CPU tensors loudly."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("red-diffeq_amd kernels run on the MI355X only (got a CPU tensor); "
                               "there is deliberately no CPU fallback")


def stream_of(t):
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def ptr(t):
    return c_void_p(t.data_ptr()) if t is not None else c_void_p(0)
