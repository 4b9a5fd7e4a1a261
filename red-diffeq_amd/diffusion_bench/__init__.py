"""diffusion_bench — the DiffusionFWI baseline of the reference (SimingShan/red-diffeq
diffusion_bench/) on the MI355X operators: the HIP FWI forward/adjoint, the HIP U-Net behind
GaussianDiffusion.p_mean_variance, the HIP L1 misfit, fused Adam and fused metrics.

ILVR_FWI adds the ILVR low-frequency conditioning (its bicubic resampler restated as per-axis
weight matrices)."""
from .diffusionfwi import DiffusionFWI, merge_patches_to_data, split_data_to_patches
from .ilvr_fwi import ILVR_FWI, resize, resize_matrix

__all__ = ["DiffusionFWI", "ILVR_FWI", "split_data_to_patches", "merge_patches_to_data", "resize", "resize_matrix"]
