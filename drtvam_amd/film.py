"""Volumetric film (mirror of drtvam/film.py).

Layout: ``data[z][y][x][c]`` fp32 with flat index ``x + y*res.x + z*res.x*res.y``
(sensor.py:405).  The reference swaps the props: ``res.x = props['resy']`` and
``res.y = props['resx']`` (film.py:10-11); kept as is.
"""
from __future__ import annotations

import torch


class VolumetricFilm:
    def __init__(self, props):
        resz = props.get('resz', 256)
        resy = props.get('resx', 256)
        resx = props.get('resy', 256)
        self.res = (resx, resy, resz)
        self.surface_aware = props.get('surface_aware', False)
        self.channels = 2 if self.surface_aware else 1
        self.data = None

    @property
    def shape(self):
        return (self.res[2], self.res[1], self.res[0], self.channels)

    def resolution(self):
        return self.res

    def clear(self, device=None):
        self.data = torch.zeros(self.shape, dtype=torch.float32, device=device)

    def develop(self):
        return self.data

    def to_string(self):
        return f'VolumetricFilm[\n    resolution = {self.shape},\n]'


films = {'vfilm': VolumetricFilm}
