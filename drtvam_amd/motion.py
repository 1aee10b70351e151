"""Projector motion models (mirror of drtvam/motion.py).

``CircularMotion.eval(t)`` returns the projector-to-world transform of
motion.py:26-36 (Mitsuba ``look_at`` from ``distance*(cos a, sin a, 0)`` towards
the origin, up = +z, a = 2*pi*t, negated when clockwise) as a 4x4 numpy
matrix.  The GPU kernels use the same rotation through per-angle (cos, sin)
tables built by the plan.
"""
from __future__ import annotations

import numpy as np


class Motion:
    """Maps a normalised time t in [0, 1] to the projector's to_world transform."""

    def __init__(self, props):
        raise NotImplementedError

    def eval(self, time):
        raise NotImplementedError


class CircularMotion(Motion):
    def __init__(self, props):
        self.distance = props['distance']
        self.tilt = props.get('tilt', 0.)  # parsed but unused, as in motion.py:22
        self.clockwise = props.get('clockwise', False)

    def angle(self, time):
        alpha = np.float32(6.2831855) * np.asarray(time, dtype=np.float32)
        return -alpha if self.clockwise else alpha

    def eval(self, time):
        alpha = float(self.angle(time))
        c, s = np.cos(alpha), np.sin(alpha)
        origin = self.distance * np.array([c, s, 0.0])
        d = -origin / np.linalg.norm(origin)
        up = np.array([0.0, 0.0, 1.0])
        left = np.cross(up, d)
        left /= np.linalg.norm(left)
        new_up = np.cross(d, left)
        m = np.eye(4)
        m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = left, new_up, d, origin
        return m


motions = {
    'circular': CircularMotion,
}
