"""Scene helpers shared by the discretisation tests (not a test module)."""
import copy
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# tests/files/double_cylindrical.json of the reference (data, restated): the hollow gear target
# at size 8 on a 14 x 14 x 1 mm sensor of 50 x 50 x 1 voxels.  The double-cylinder vial is out of
# scope and irrelevant to the discretisation, so an index-matched vial
# stands in for it.
DOUBLE_CYLINDRICAL_GEAR = {
    "vial": {"type": "index_matched", "r": 7, "medium": {"ior": 1.48, "extinction": 0.05, "albedo": 0.0}},
    "projector": {"type": "collimated", "n_patterns": 200, "resx": 200, "resy": 10, "pixel_size": 75e-3,
                  "motion": "circular", "distance": 20},
    "sensor": {"type": "dda", "scalex": 14, "scaley": 14, "scalez": 1,
               "film": {"type": "vfilm", "resx": 50, "resy": 50, "resz": 1}},
    "target": {"filename": os.path.join(GOLDEN, "hollow_gear.ply"), "size": 8.0},
    "loss": {"type": "threshold", "tl": 0.6, "tu": 0.85},
}


def scene_of(cfg):
    from drtvam_amd.optimize import load_scene
    from drtvam_amd.scene import load_dict
    cfg = copy.deepcopy(cfg)
    cfg["projector"]["device"] = "cpu"
    scene = load_dict(load_scene(cfg))
    return scene, scene.sensor_by_id("sensor")


def grid_desc(scene, sensor):
    """A tvam_desc carrying the sensor grid and the target's world-space triangles."""
    from drtvam_amd import _abi
    from drtvam_amd.utils import target_triangles
    d = _abi.TvamDesc()
    _abi.load_library().tvam_desc_init(d)
    d.film_res[:] = sensor.resolution()
    d.bbox_min[:] = [float(v) for v in sensor.bbox_min]
    d.bbox_max[:] = [float(v) for v in sensor.bbox_max]
    d.set_target(target_triangles(scene))
    return d


def gear_fixture():
    """tests/files/target_hollow_gear.npy of the reference: its discretize() output for the
    hollow gear (shape (1, 50, 50, 1), 188 voxels inside), produced by Mitsuba."""
    return np.load(os.path.join(GOLDEN, "target_hollow_gear.npy"))


def box_hole_reference():
    """The voxelised reference of tests/test_optimization.py:130-144 (reference test data, restated)."""
    reference = np.zeros((50, 100, 100))
    reference[5:45, 10:90, 10:90] = 1
    y, x = np.meshgrid(np.arange(100), np.arange(100))
    mask = (x - 50) ** 2 + (y - 30) ** 2 < (20 + 0.5) ** 2
    array = np.zeros((50, 100, 100), dtype=int)
    array[5:45, mask] = 1
    return reference - array
