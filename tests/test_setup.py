"""Setup-side pieces around the hot path: scene assembly (discretisation: test_discretize.py)."""
import os

import numpy as np
import pytest

from drtvam_amd.configs import BOX_HOLE_INDEX_MATCHED, desc_from_config

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_box_hole_desc_follows_config():
    d = desc_from_config(BOX_HOLE_INDEX_MATCHED)
    assert list(d.film_res) == [100, 100, 50]
    assert d.bbox_min[0] == pytest.approx(-2.5) and d.bbox_max[2] == pytest.approx(0.625)
    assert d.n_patterns == 200 and d.res_x == 200 and d.res_y == 20
    assert d.vial_r == pytest.approx(2.9) and d.sigma_t == pytest.approx(0.03)
    assert d.pixel_size_x == pytest.approx(0.05)


def test_film_resolution_swap():
    """film.py:9-11: res.x = props['resy'], res.y = props['resx']."""
    from drtvam_amd.film import VolumetricFilm
    f = VolumetricFilm({'resx': 10, 'resy': 20, 'resz': 30})
    assert f.resolution() == (20, 10, 30)
    assert f.shape == (30, 10, 20, 1)


def test_cuboid_triangles_outward():
    """The analytic target's Radon-filter mesh: 12 triangles, outward normals, covering the box."""
    from drtvam_amd.utils import cuboid_triangles
    lo, hi = np.array([-1.0, 0.0, 2.0]), np.array([1.0, 3.0, 2.5])
    t = cuboid_triangles(lo, hi).astype(np.float64)
    assert t.shape == (12, 3, 3)
    n = np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0])
    assert np.all(np.einsum('ij,ij->i', n, t.mean(axis=1) - 0.5 * (lo + hi)) > 0)
    area = 0.5 * np.linalg.norm(n, axis=1).sum()
    e = hi - lo
    assert np.isclose(area, 2 * (e[0] * e[1] + e[1] * e[2] + e[0] * e[2]))
