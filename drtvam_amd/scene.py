"""Scene assembly and the ``render`` / ``traverse`` entry points.

Mirrors the pieces of Mitsuba that drtvam relies on around the hot path:
``load_dict`` (optimize.py:90), ``traverse`` (optimize.py:91, the
'projector.active_data' / 'projector.active_pixels' parameters) and
``render(scene, params, integrator, sensor, spp, spp_grad, seed)``
(optimize.py:216, :294, :328).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .geometry import CylindricalVial, IndexMatchedVial, Container
from .integrators import integrators, VolumeIntegrator
from .projector import TVAMProjector, emitters
from .sensor import VolumetricSensor, sensors


class Scene:
    def __init__(self):
        self.projector: Optional[TVAMProjector] = None
        self.n_projectors = 0
        self._sensors: list[tuple[str, VolumetricSensor]] = []
        self.container: Optional[Container] = None
        self.target = None
        self.integrator = None
        self.shapes = {}

    def emitters(self):
        return [self.projector] if self.projector is not None else []

    def sensors(self):
        return [s for _, s in self._sensors]

    def sensor_by_id(self, sid):
        for k, s in self._sensors:
            if k == sid:
                return s
        raise KeyError(sid)

    def sensor_ids(self):
        return [k for k, _ in self._sensors]


def _medium_from(d, ior):
    m = {'ior': ior, 'extinction': d.get('sigma_t', 1.0), 'albedo': d.get('albedo', 0.0)}
    if 'phase' in d:
        m['phase'] = d['phase']
    return m


def _container_from_shapes(scene_dict):
    media = {k: v for k, v in scene_dict.items() if isinstance(v, dict) and v.get('type') == 'homogeneous'}
    shapes = {k: v for k, v in scene_dict.items() if isinstance(v, dict) and v.get('type') in ('cylinder', 'cube', 'ply')}
    holder = [(k, v) for k, v in shapes.items() if 'interior' in v]
    if not holder:
        return None
    if len(holder) > 1:
        raise ValueError("There is more than one medium in the scene. Only one is supported")
    name, shp = holder[0]
    interior = shp['interior']
    if interior.get('type') == 'ref':
        interior = media[interior['id']]
    bsdf = shp.get('bsdf', {'type': 'diffuse'})
    if shp['type'] == 'cylinder' and bsdf.get('type') == 'null':
        p0, p1 = np.asarray(shp.get('p0', [0, 0, 0]), float), np.asarray(shp.get('p1', [0, 0, 1]), float)
        if abs(p0[0]) + abs(p0[1]) + abs(p1[0]) + abs(p1[1]) > 0 or abs(p0[2] + p1[2]) > 1e-9:
            raise NotImplementedError("only vials centred on the z axis are supported")
        return IndexMatchedVial({'r': shp['radius'], 'height': float(abs(p1[2] - p0[2])),
                                 'medium': _medium_from(interior, 1.0)})
    if shp['type'] == 'cylinder' and bsdf.get('type') == 'dielectric':
        outer = [v for k, v in shapes.items() if k != name and v['type'] == 'cylinder']
        if len(outer) == 1:
            p0, p1 = np.asarray(shp['p0'], float), np.asarray(shp['p1'], float)
            return CylindricalVial({'r_int': shp['radius'], 'r_ext': outer[0]['radius'],
                                    'height': float(abs(p1[2] - p0[2])),
                                    'ior': bsdf.get('ext_ior', 1.5),
                                    'medium': _medium_from(interior, bsdf.get('int_ior', 1.0))})
    raise NotImplementedError(f"container shape '{name}' is not supported by the GPU engine")


def load_dict(scene_dict: dict) -> Scene:
    """Instantiate the plugins of a scene dictionary (Mitsuba ``load_dict`` for the TVAM plugin set)."""
    if scene_dict.get('type', 'scene') != 'scene':
        raise ValueError("expected a dictionary of type 'scene'")
    scene = Scene()
    for key, v in scene_dict.items():
        if key == 'type':
            continue
        if isinstance(v, TVAMProjector):
            scene.projector = v
            scene.n_projectors += 1
            continue
        if isinstance(v, VolumetricSensor):
            scene._sensors.append((key, v))
            continue
        if not isinstance(v, dict) or 'type' not in v:
            continue
        t = v['type']
        if t in emitters:
            scene.projector = emitters[t](v)
            scene.n_projectors += 1
        elif t in sensors:
            scene._sensors.append((key, sensors[t](v)))
        elif t in integrators:
            scene.integrator = integrators[t](v)
        else:
            scene.shapes[key] = v
    scene.container = scene_dict.get('_container') or _container_from_shapes(scene_dict)
    scene.target = scene_dict.get('target')
    if scene.integrator is None:
        scene.integrator = VolumeIntegrator({})
    return scene


class SceneParameters(dict):
    """``mi.traverse(scene)`` equivalent for the differentiable projector data."""

    def __init__(self, scene: Scene):
        super().__init__()
        self.scene = scene
        p = scene.projector
        dict.__setitem__(self, 'projector.active_data', p.active_data)
        dict.__setitem__(self, 'projector.active_pixels', p.active_pixels)

    def update(self, values=None):
        if values is not None:
            for k in ('projector.active_data', 'projector.active_pixels'):
                if k in values:
                    dict.__setitem__(self, k, values[k])
        self.scene.projector.set_active(self['projector.active_data'], self['projector.active_pixels'])


def traverse(scene: Scene) -> SceneParameters:
    return SceneParameters(scene)


def render(scene: Scene, params=None, integrator=None, sensor=0, spp: int = 0, spp_grad: int = 0, seed: int = 0,
           seed_grad: Optional[int] = None) -> torch.Tensor:
    """Differentiable render (``mi.render``): gradients flow to projector.active_data when it requires grad."""
    integrator = integrator or scene.integrator
    x = scene.projector.active_data
    if x.requires_grad and torch.is_grad_enabled():
        return integrator.render_differentiable(scene, sensor, spp=spp, spp_grad=spp_grad or None, seed=seed,
                                                seed_grad=seed_grad)
    return integrator.render(scene, sensor, seed=seed, spp=spp)
