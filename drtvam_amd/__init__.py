"""drtvam_amd — MI355X-native TVAM forward/adjoint projection engine.

Drop-in for Dr.TVAM's hot path (the `volume` integrator + `dda` sensor +
`vfilm` film + `collimated` projector ray march) behind the same plugin
names, registries, loss interface and optimizer.  The ray march runs in the
hand-written gfx950 HIP kernels of libtvam.so (include/tvam.h); there is no
CPU fallback.
"""
from . import geometry, motion, loss
from .film import VolumetricFilm
from .geometry import Container, IndexMatchedVial, CylindricalVial, SquareVial, CustomVial, DoubleCylindricalVial
from .integrators import VolumeIntegrator, TVAMIntegrator
from .lbfgs import LinearLBFGS
from .loss import Loss, L2Loss, ThresholdedLoss
from .motion import Motion, CircularMotion
from .projector import TVAMProjector, CollimatedProjector, TelecentricProjector, LensProjector
from .scene import load_dict, render, traverse, Scene
from .sensor import VolumetricSensor, DDAVolumetricSensor, RatioVolumetricSensor, DeltaVolumetricSensor

__version__ = "0.1.0"


def register_geometry(name, cls):
    if name in geometry.geometries:
        raise ValueError(f"Geometry '{name}' is already registered.")
    if not issubclass(cls, geometry.Container):
        raise ValueError(f"Class '{cls}' is not a subclass of 'geometry.Container'.")
    geometry.geometries[name] = cls


def register_motion(name, cls):
    if name in motion.motions:
        raise ValueError(f"Motion '{name}' is already registered.")
    if not issubclass(cls, motion.Motion):
        raise ValueError(f"Class '{cls}' is not a subclass of 'motion.Motion'.")
    motion.motions[name] = cls


def register_loss(name, cls):
    if name in loss.losses:
        raise ValueError(f"Loss '{name}' is already registered.")
    if not issubclass(cls, loss.Loss):
        raise ValueError(f"Class '{cls}' is not a subclass of 'loss.Loss'.")
    loss.losses[name] = cls
