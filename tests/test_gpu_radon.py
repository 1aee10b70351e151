"""GPU parity of the Radon filter (tvam_radon) against the oracle, and the filtered active set."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config, square_vial
from drtvam_amd.engine import Projection
from drtvam_amd.utils import read_ply

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def tris(name):
    v, f = read_ply(os.path.join(GOLDEN, name))
    return np.asarray(v, np.float32)[np.asarray(f)]


def box_hole_target():
    # tests/files/box_hole.ply scaled to size 4 (optimize.py:30-50)
    from drtvam_amd.utils import mesh_bbox, target_transform
    lo, hi = mesh_bbox(os.path.join(GOLDEN, "box_hole.ply"))
    m = target_transform(lo, hi, 4.0)
    t = tris("box_hole.ply").astype(np.float64)
    return (t @ m[:3, :3].T + m[:3, 3]).astype(np.float32)


SCENES = {
    "index_matched": lambda **k: benchy_index_matched(N=24, angles=10, size_mm=5.0, r=2.9, **k),
    "cylindrical": lambda **k: cylindrical_refraction(N=24, angles=10, size_mm=5.0, r_int=3.5, r_ext=4.0, **k),
    "square": lambda **k: square_vial(N=24, angles=10, **k),
}


@pytest.mark.parametrize("vial", list(SCENES))
@pytest.mark.parametrize("target", ["box", "box_hole"])
def test_radon_matches_oracle(oracle, vial, target):
    d = desc_from_config(SCENES[vial](regular_sampling=False, spp=4))
    t = tris("occlusion.ply") if target == "box" else box_hole_target()
    ref = oracle.radon(d, t, spp=4, seed=0, max_depth=5, nthreads=8)
    got = Projection(d, "cuda:0").radon(t, spp=4, seed=0, max_depth=5).cpu().numpy()
    assert (ref > 0).sum() > 0
    mism = np.sum((ref > 0) != (got > 0))
    assert mism <= max(1, 1e-3 * ref.size)
    assert np.linalg.norm(got - ref) <= 1e-4 * np.linalg.norm(ref)
