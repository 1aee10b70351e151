"""Volumetric sensors (mirror of drtvam/sensor.py).

The sensor defines the voxel grid: ``bbox = to_world @ [-0.5, 0.5]^3``
(sensor.py:14-16) and ``voxel_size = extents / film resolution`` (:19).  The
DDA accumulation itself (:306-440) runs inside the HIP kernels; the sensor
contributes the grid to the plan descriptor.
"""
from __future__ import annotations

import numpy as np

from .film import VolumetricFilm, films
from . import _abi


def _as_transform(t):
    if t is None:
        return np.eye(4)
    t = np.asarray(t, dtype=np.float64)
    if t.shape == (4, 4):
        return t
    if t.shape == (3,):
        return np.diag([t[0], t[1], t[2], 1.0])
    raise ValueError("to_world must be a 4x4 matrix or a scale triple")


class VolumetricSensor:
    def __init__(self, props):
        film = props.get('film', {'type': 'vfilm'})
        if isinstance(film, dict):
            ftype = film.get('type', 'vfilm')
            if ftype not in films:
                raise ValueError("Tried to load a VolumetricSensor with a non-volumetric film. The film must be of type VolumetricFilm.")
            film = films[ftype](film)
        if not isinstance(film, VolumetricFilm):
            raise ValueError("Tried to load a VolumetricSensor with a non-volumetric film. The film must be of type VolumetricFilm.")
        self.m_film = film
        self.to_world = _as_transform(props.get('to_world', None))
        lin, off = self.to_world[:3, :3], self.to_world[:3, 3]
        if np.count_nonzero(lin - np.diag(np.diag(lin))):
            raise ValueError("only axis-aligned (scale + translate) sensor transforms are supported")
        c0 = (lin @ np.full(3, -0.5) + off).astype(np.float32)
        c1 = (lin @ np.full(3, 0.5) + off).astype(np.float32)
        self.bbox_min = np.minimum(c0, c1)
        self.bbox_max = np.maximum(c0, c1)
        res = np.array(self.m_film.resolution(), dtype=np.float32)
        self.voxel_size = (self.bbox_max - self.bbox_min) / res  # fp32, sensor.py:19
        self.volumes = None

    def film(self):
        return self.m_film

    def resolution(self):
        return self.m_film.resolution()

    def compute_volume(self, scene=None, sample_count=2 ** 14):
        """Voxel volume (sensor.py:47-51), or for a surface-aware film the volumes [Z, Y, X, 2]
        inside / outside the scene's target mesh (sensor.py:53-110, cached like the reference),
        estimated on the GPU (tvam_compute_volume)."""
        if not self.m_film.surface_aware:
            return float(np.prod(self.voxel_size, dtype=np.float32))
        if self.volumes is not None:
            return self.volumes
        if scene is None or scene.target is None:
            raise ValueError("No target shape found in the scene")
        from .integrators.common import TVAMIntegrator
        from .engine import Projection
        d = TVAMIntegrator({}).desc(scene, self)
        proj = Projection(d, scene.projector.device)
        self.volumes = proj.compute_volume(sample_count)
        proj.close()
        return self.volumes

    def fill_desc(self, desc: _abi.TvamDesc) -> None:
        for a in range(3):
            desc.bbox_min[a] = float(self.bbox_min[a])
            desc.bbox_max[a] = float(self.bbox_max[a])
            desc.film_res[a] = int(self.m_film.res[a])
        desc.film_channels = self.m_film.channels


class DDAVolumetricSensor(VolumetricSensor):
    """Analytic per-voxel absorption by grid traversal (sensor.py:297-440)."""

    def fill_desc(self, desc):
        super().fill_desc(desc)
        desc.sensor_type = _abi.SENSOR_DDA


class RatioVolumetricSensor(VolumetricSensor):
    """Ratio-tracking estimator (sensor.py:193-295): deposits at points stepped by a majorant
    along every medium segment (the general per-path kernel)."""

    def __init__(self, props):
        super().__init__(props)
        self.majorant = props['majorant']

    def to_string(self):
        return f'RatioVolumetricSensor[\n    majorant = {self.majorant},\n]'

    def fill_desc(self, desc):
        super().fill_desc(desc)
        desc.sensor_type = _abi.SENSOR_RATIO
        desc.majorant = float(self.majorant)


class DeltaVolumetricSensor(VolumetricSensor):
    """Collision estimator (sensor.py:112-191): deposits at the medium interactions of
    scattering media (the general per-path kernel)."""

    def to_string(self):
        return 'DeltaVolumetricSensor[]'

    def fill_desc(self, desc):
        super().fill_desc(desc)
        desc.sensor_type = _abi.SENSOR_DELTA


sensors = {
    'delta': DeltaVolumetricSensor,
    'ratio': RatioVolumetricSensor,
    'dda': DDAVolumetricSensor,
}
