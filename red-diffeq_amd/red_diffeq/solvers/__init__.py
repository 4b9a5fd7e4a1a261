from .pde import FWIForward

__all__ = ["FWIForward"]
