"""red_diffeq — MI355X-native implementation of red-diffeq's inversion hot path.

Drop-in for the reference package's public API (SimingShan/red-diffeq red_diffeq/__init__.py):
the 2-D acoustic FWI forward/adjoint, the L1 misfit and TV/Tikhonov regularisers run as
hand-written HIP kernels (libred_diffeq_hip.so, C ABI in include/red_diffeq_fwi.h).
"""
__version__ = "0.1.0"

from .config import get_config, get_marmousi_config, load_config, print_config, save_config, update_config
from .core.inversion import InversionEngine
from .models.diffusion import GaussianDiffusion, Unet
from .regularization.base import RegularizationMethod
from .regularization.benchmark import tikhonov_loss, total_variation_loss
from .regularization.diffusion import RED_DiffEq, RED_DiffEq_POST_PROCESS
from .solvers.pde import FWIForward
from .utils.data_trans import prepare_initial_model, s_normalize_none, v_denormalize, v_normalize
from .utils.seed_utils import SeedContext, get_rng_state, set_rng_state, set_seed, worker_init_fn
from .utils.ssim import SSIM

__all__ = ["get_config", "get_marmousi_config", "load_config", "save_config", "update_config", "print_config",
           "InversionEngine", "GaussianDiffusion", "Unet", "FWIForward", "RED_DiffEq", "RED_DiffEq_POST_PROCESS",
           "total_variation_loss", "tikhonov_loss", "RegularizationMethod", "prepare_initial_model",
           "v_denormalize", "v_normalize", "s_normalize_none", "SSIM", "set_seed", "SeedContext",
           "get_rng_state", "set_rng_state", "worker_init_fn"]
