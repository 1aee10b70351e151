"""TVAM integrator base (mirror of drtvam/integrators/common.py).

Holds the integrator properties of common.py:6-22 plus max_depth / rr_depth,
and turns (scene, sensor, integrator) into the C descriptor of libtvam.so.
Plans are cached per (descriptor, device): building one is the analogue of
Dr.Jit tracing + compiling the megakernel, done once per configuration.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _abi


class TVAMIntegrator:
    def __init__(self, props):
        props = dict(props)
        self.max_depth = props.get('max_depth', 6)
        self.rr_depth = props.get('rr_depth', 5)
        self.sample_time = props.get('sample_time', False)
        self.print_time = props.get('print_time', 1.)
        self.target_id = props.get('target_id', 'target')
        self.transmission_only = props.get('transmission_only', True)
        self.regular_sampling = props.get('regular_sampling', False)
        self.angle_range = props.get('angle_range', None)  # (begin, end): angle shard of this rank
        self.row_band = props.get('row_band', None)  # (begin, end): crop rows of this rank (z-slab sharding)
        self.slab = props.get('slab', None)          # (begin, end): film z-slices of this rank
        self.tile = props.get('tile', 0)
        self.flags = props.get('flags', 0)
        self._plans = {}

    def parse_scene(self, scene):
        if scene.container is None:
            raise ValueError("No printing medium found in the scene")
        return scene.container, scene.target

    def desc(self, scene, sensor) -> _abi.TvamDesc:
        d = _abi.default_desc()
        projector = scene.projector
        projector.fill_desc(d)
        sensor.fill_desc(d)
        scene.container.fill_desc(d)
        d.print_time = float(self.print_time)
        d.regular_sampling = int(bool(self.regular_sampling))
        d.sample_time = int(bool(self.sample_time))
        d.max_depth = int(self.max_depth)
        d.rr_depth = int(self.rr_depth)
        d.transmission_only = int(bool(self.transmission_only))
        if self.angle_range is not None:
            d.angle_begin, d.angle_end = int(self.angle_range[0]), int(self.angle_range[1])
        if self.row_band is not None:
            r0, r1 = int(self.row_band[0]), int(self.row_band[1])
            d.crop_offset_y += r0
            d.crop_y = r1 - r0
        if self.slab is not None:
            d.slab_begin, d.slab_end = int(self.slab[0]), int(self.slab[1])
        d.tile = int(self.tile)
        d.flags = int(self.flags)
        if sensor.film().surface_aware:  # the target mesh stays in the scene (optimize.py:188-191)
            from ..utils import target_triangles
            d.set_target(target_triangles(scene))
        return d

    def projection(self, scene, sensor, device=None):
        from ..engine import Projection
        d = self.desc(scene, sensor)
        dev = torch.device(device) if device is not None else scene.projector.device
        key = (bytes(memoryview(ctypes.string_at(ctypes.addressof(d), ctypes.sizeof(d)))), str(dev))
        proj = self._plans.get(key)
        if proj is None:
            proj = Projection(d, dev)
            if sensor.film().surface_aware:  # inv_vol of the two channels (volume.py:41-42)
                proj.set_volumes(sensor.compute_volume(scene).to(dev))
            self._plans[key] = proj
        return proj

    def prepare(self, projector, seed: int = 0, spp: int = 0):
        """Effective spp (common.py:41-68): regular sampling forces 1, spp=0 uses the sampler's count (4)."""
        if self.regular_sampling:
            spp = 1
        if spp == 0:
            spp = int(projector.sampler().get('sample_count', 4)) if isinstance(projector.sampler(), dict) else 4
        wavefront_size = projector.active_size() * spp
        if wavefront_size > 2 ** 32:
            raise Exception(
                "The total number of Monte Carlo samples required by this "
                "rendering task (%i) exceeds 2^32 = 4294967296. Please use "
                "fewer samples per pixel or render using multiple passes."
                % wavefront_size)
        return seed, spp
