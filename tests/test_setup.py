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
