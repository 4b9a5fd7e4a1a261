from .diffusion import GaussianDiffusion, Unet

__all__ = ["GaussianDiffusion", "Unet"]
