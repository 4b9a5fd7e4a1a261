from .base import RegularizationMethod
from .benchmark import tikhonov_loss, total_variation_loss
from .diffusion import RED_DiffEq, RED_DiffEq_POST_PROCESS

__all__ = ["RED_DiffEq", "RED_DiffEq_POST_PROCESS", "total_variation_loss", "tikhonov_loss",
           "RegularizationMethod"]
