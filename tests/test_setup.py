"""Setup-side pieces around the hot path: PLY target discretisation and scene assembly."""
import os

import numpy as np
import pytest

from drtvam_amd.configs import BOX_HOLE_INDEX_MATCHED, desc_from_config

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def box_hole_reference():
    """The voxelised reference of tests/test_optimization.py:130-144 (reference test data, restated)."""
    reference = np.zeros((50, 100, 100))
    reference[5:45, 10:90, 10:90] = 1
    y, x = np.meshgrid(np.arange(100), np.arange(100))
    mask = (x - 50) ** 2 + (y - 30) ** 2 < (20 + 0.5) ** 2
    array = np.zeros((50, 100, 100), dtype=int)
    array[5:45, mask] = 1
    return reference - array


def test_discretize_box_hole_matches_reference_voxelisation():
    import copy
    from drtvam_amd.optimize import load_scene
    from drtvam_amd.scene import load_dict
    from drtvam_amd.utils import discretize

    cfg = copy.deepcopy(BOX_HOLE_INDEX_MATCHED)
    cfg["target"]["filename"] = os.path.join(GOLDEN, "box_hole.ply")
    cfg["projector"]["device"] = "cpu"
    scene = load_dict(load_scene(cfg))
    occ = discretize(scene, sensor=scene.sensor_by_id("sensor")).numpy()[..., 0]
    assert occ.shape == (50, 100, 100)
    ref = box_hole_reference()
    # box extents match exactly; the only disagreement is the ring of voxel centres lying exactly on
    # the hole surface (radius 20 voxels): the analytic array counts radius < 20.5 as hole, the
    # inscribed polygonal mesh does not (~0.84 % of the grid)
    for ax in range(3):
        other = tuple(a for a in range(3) if a != ax)
        assert (np.nonzero(occ.sum(axis=other))[0][[0, -1]] == np.nonzero(ref.sum(axis=other))[0][[0, -1]]).all()
    agree = np.mean(occ == ref)
    assert agree > 0.994, agree


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
