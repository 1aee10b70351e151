"""End-to-end optimisation on the GPU, restating tests/test_optimization.py:104-155 of the
reference for the index-matched box-with-hole config (tests/files/box_hole_index_matched.json):
after the optimisation, > 99.4 % of the voxels thresholded at (tl + tu) / 2 must match the
voxelised reference of test_optimization.py:130-144.  The cylindrical config
(tests/files/box_hole_cylindrical.json) runs as given (scattering resin, albedo 0.5, Rayleigh)
and with its albedo set to 0."""
import copy
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd.configs import BOX_HOLE_CYLINDRICAL, BOX_HOLE_INDEX_MATCHED
from drtvam_amd.optimize import optimize

import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_setup import box_hole_reference  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_box_hole_index_matched_optimization(tmp_path):
    cfg = copy.deepcopy(BOX_HOLE_INDEX_MATCHED)
    cfg["target"]["filename"] = os.path.join(GOLDEN, "box_hole.ply")
    cfg["output"] = str(tmp_path)
    vol = optimize(cfg, device="cuda:0")
    vol = vol.cpu().numpy()[..., 0]
    th = (cfg["loss"]["tl"] + cfg["loss"]["tu"]) / 2
    correct = np.mean(np.isclose(box_hole_reference(), vol > th)) * 100
    print("percentage correct", correct)
    assert correct > 99.4
    loss = np.load(tmp_path / "loss.npy")
    assert loss[-1] < 0.05 * loss[0]
    assert (tmp_path / "patterns.npz").exists() and (tmp_path / "final.npy").exists()


@pytest.mark.parametrize("albedo", [0.5, 0.0])
def test_box_hole_cylindrical_optimization(tmp_path, albedo):
    cfg = copy.deepcopy(BOX_HOLE_CYLINDRICAL)
    cfg["vial"]["medium"]["albedo"] = albedo  # 0.5: the reference file; 0: non-scattering variant
    cfg["target"]["filename"] = os.path.join(GOLDEN, "box_hole.ply")
    cfg["output"] = str(tmp_path)
    vol = optimize(cfg, device="cuda:0")
    vol = vol.cpu().numpy()[..., 0]
    th = (cfg["loss"]["tl"] + cfg["loss"]["tu"]) / 2
    correct = np.mean(np.isclose(box_hole_reference(), vol > th)) * 100
    print("percentage correct", correct)
    assert correct > 99.4
    loss = np.load(tmp_path / "loss.npy")
    assert loss[-1] < 0.05 * loss[0]
