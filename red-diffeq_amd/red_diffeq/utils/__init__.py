from .data_trans import (v_normalize, v_denormalize, s_normalize, s_denormalize, s_normalize_none,
                         add_noise_to_seismic, missing_trace, prepare_initial_model)
from .ssim import SSIM, ssim

__all__ = ["v_normalize", "v_denormalize", "s_normalize", "s_denormalize", "s_normalize_none",
           "add_noise_to_seismic", "missing_trace", "prepare_initial_model", "SSIM", "ssim"]
