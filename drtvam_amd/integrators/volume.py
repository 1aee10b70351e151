"""Volume integrator (mirror of drtvam/integrators/volume.py).

``render`` = VolumeIntegrator.render (volume.py:18-56): one forward
projection (HIP tile kernel) returning the dose tensor [Z, Y, X, C].
``render_backward`` = volume.py:97-134: the adjoint projection of ``grad_in``
accumulated into ``projector.active_data.grad``.
"""
from __future__ import annotations

from typing import Optional

import torch

from .common import TVAMIntegrator
from ..engine import derive_seed_grad, render as engine_render


def _check_projectors(scene):
    if scene.projector is None:
        raise Exception("No projector found in the scene")
    if getattr(scene, 'n_projectors', 1) > 1:
        raise Exception("The scene contains more than one projector. Only one is supported")


class VolumeIntegrator(TVAMIntegrator):

    def to_string(self):
        return ('VolumeIntegrator[\n'
                f'    self.print_time={self.print_time},\n'
                f'    self.transmission_only={self.transmission_only},\n'
                f'    self.sample_time={self.sample_time},\n'
                f'    self.max_depth={self.max_depth},\n'
                f'    self.rr_depth={self.rr_depth},\n'
                ']')

    def _sensor(self, scene, sensor):
        if isinstance(sensor, int):
            return scene.sensors()[sensor]
        if isinstance(sensor, str):
            return scene.sensor_by_id(sensor)
        return sensor

    def render(self, scene, sensor=0, seed: int = 0, spp: int = 0, develop: bool = True,
               evaluate: bool = True) -> torch.Tensor:
        _check_projectors(scene)
        sensor = self._sensor(scene, sensor)
        projector = scene.projector
        seed, spp = self.prepare(projector, seed, spp)
        proj = self.projection(scene, sensor)
        pix = None if projector.dense else projector.active_pixels
        with torch.no_grad():
            dose = proj.forward(projector.active_data.detach().contiguous(), pix, spp, seed)
        sensor.film().data = dose
        return dose

    def render_differentiable(self, scene, sensor=0, spp: int = 0, spp_grad: Optional[int] = None, seed: int = 0,
                              seed_grad: Optional[int] = None, active_data: Optional[torch.Tensor] = None):
        """mi.render with AD: dose depends differentiably on active_data (default: projector.active_data)."""
        _check_projectors(scene)
        sensor = self._sensor(scene, sensor)
        projector = scene.projector
        seed, spp = self.prepare(projector, seed, spp)
        spp_grad = spp if not spp_grad else (1 if self.regular_sampling else spp_grad)
        proj = self.projection(scene, sensor)
        pix = None if projector.dense else projector.active_pixels
        x = projector.active_data if active_data is None else active_data
        return engine_render(proj, x, pix, spp, spp_grad, seed, derive_seed_grad(seed) if seed_grad is None else seed_grad)

    def render_forward(self, scene, params=None, sensor=0, seed: int = 0, spp: int = 0,
                       tangent: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Forward-mode derivative (volume.py:58-95): the dose tangent [Z, Y, X, C] produced by a
        tangent of projector.active_data.  The render is linear in the patterns, so this is the
        forward projection of the tangent (the reference propagates dr.grad(active_data) through
        Le in ADMode.Forward and scales by inv_vol, as the forward kernel does).  `tangent`
        defaults to projector.active_data.grad, the slot the reference reads it from."""
        _check_projectors(scene)
        sensor = self._sensor(scene, sensor)
        projector = scene.projector
        if tangent is None:
            tangent = projector.active_data.grad
        if tangent is None:
            raise ValueError("render_forward: no tangent (set projector.active_data.grad or pass `tangent`)")
        if tangent.numel() != projector.active_size():
            raise ValueError("render_forward: the tangent must have one entry per active pixel")
        seed, spp = self.prepare(projector, seed, spp)
        proj = self.projection(scene, sensor)
        pix = None if projector.dense else projector.active_pixels
        with torch.no_grad():
            return proj.forward(tangent.detach().to(dtype=torch.float32).contiguous(), pix, spp, seed)

    def render_backward(self, scene, params, grad_in: torch.Tensor, sensor=0, seed: int = 0, spp: int = 0) -> None:
        _check_projectors(scene)
        sensor = self._sensor(scene, sensor)
        projector = scene.projector
        seed, spp = self.prepare(projector, seed, spp)
        proj = self.projection(scene, sensor)
        pix = None if projector.dense else projector.active_pixels
        g = proj.adjoint(grad_in.contiguous(), projector.active_size(), pix, spp, seed)
        x = projector.active_data
        if x.grad is None:
            x.grad = g
        else:
            x.grad += g


integrators = {'volume': VolumeIntegrator}
