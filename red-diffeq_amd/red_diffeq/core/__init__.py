from .inversion import InversionEngine
from .losses import LossCalculator
from .metrics import MetricsCalculator

__all__ = ["InversionEngine", "MetricsCalculator", "LossCalculator"]
