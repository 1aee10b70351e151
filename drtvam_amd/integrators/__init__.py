from .common import TVAMIntegrator
from .volume import VolumeIntegrator, integrators

__all__ = ["TVAMIntegrator", "VolumeIntegrator", "integrators"]
