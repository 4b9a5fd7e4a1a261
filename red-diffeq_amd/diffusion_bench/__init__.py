"""diffusion_bench — the DiffusionFWI baseline of the reference (SimingShan/red-diffeq
diffusion_bench/) on the MI355X operators: the HIP FWI forward/adjoint, the HIP U-Net behind
GaussianDiffusion.p_mean_variance, the HIP L1 misfit, fused Adam and fused metrics.

ILVR_FWI (diffusion_bench/ilvr_fwi.py, with its Resizer) is not provided."""
from .diffusionfwi import DiffusionFWI, merge_patches_to_data, split_data_to_patches

__all__ = ["DiffusionFWI", "split_data_to_patches", "merge_patches_to_data"]
