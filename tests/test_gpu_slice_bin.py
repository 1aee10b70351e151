"""GPU: the 16-byte pattern binning of the voxel-driven forward (tvam_slice_bin4_kernel) against
the one-float-per-thread kernel (TVAM_SLICE_BIN1=1, read once per process: two child processes):
the same sums in the same order, so the forwards are bit-identical — index-matched and refracted
scenes, one DMD row per slice and two rows per slice (a DMD twice as fine as the film)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config
from drtvam_amd.engine import Projection
scene, N, rows = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
cfg = (benchy_index_matched if scene == "im" else cylindrical_refraction)(N=N, angles=20)
if rows != N:  # a DMD `rows / N` times as fine as the film (same extent): several rows per slice
    cfg["projector"]["resx"] = cfg["projector"]["resy"] = rows
    cfg["projector"]["pixel_size"] = cfg["projector"]["pixel_size"] * N / rows
d = desc_from_config(cfg)
p = Projection(d, "cuda:0")
n = int(d.crop_x) * int(d.crop_y) * 20
x = torch.as_tensor(np.random.default_rng(7).uniform(0, 1, n).astype(np.float32), device="cuda:0")
np.save(sys.argv[5], p.forward(x, None, 1, 0).cpu().numpy())
"""


@pytest.mark.parametrize("scene,N,rows", [("im", 96, 96), ("im", 96, 192), ("cyl", 96, 96)])
def test_vec4_binning_bit_identical(tmp_path, scene, N, rows):
    outs = []
    for knob in ("0", "1"):
        f = str(tmp_path / f"f{knob}.npy")
        env = dict(os.environ, TVAM_SLICE_BIN1=knob, TVAM_EXPERIMENTAL="1")
        r = subprocess.run([sys.executable, "-c", CHILD, ROOT, scene, str(N), str(rows), f], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(np.load(f))
    assert outs[0].shape == outs[1].shape and float(np.abs(outs[1]).max()) > 0
    assert np.array_equal(outs[0], outs[1])
