"""The reference's projector / film edge cases on the HIP path (through tvam_forward /
tvam_adjoint), against the oracle at 1e-4 relative L2:

  * the crop of tests/test_projector.py:7-38 (20 x 10 DMD, 4 x 4 crop at (8, 3), 1 mm pixels,
    distance 20): every ray of the crop has |o.y|, |o.z| < 2, so the dose vanishes outside the
    |z| < 2 slab and the forward / adjoint match the oracle;
  * `clockwise` circular motion (motion.py:23-36: the angle negated);
  * a film with resx != resy (film.py:9-11 swaps them: res.x = props['resy']).
Each runs on the planar path (regular sampling) and on the per-ray tile kernels (jittered).
"""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd.configs import benchy_index_matched, desc_from_config
from drtvam_amd.engine import Projection
from parity_util import RTOL, rel_l2

DEV = "cuda:0"


def crop_config(regular):
    cfg = benchy_index_matched(N=24, angles=12, size_mm=6.0, r=5.0, sigma_t=0.05, regular_sampling=regular,
                               spp=1 if regular else 4)
    cfg["projector"].update({"n_patterns": 12, "resx": 20, "resy": 10, "cropx": 4, "cropy": 4, "crop_offset_x": 8,
                             "crop_offset_y": 3, "pixel_size": 1.0, "distance": 20.0})
    return cfg


def clockwise_config(regular):
    cfg = benchy_index_matched(N=32, angles=24, regular_sampling=regular, spp=1 if regular else 3)
    cfg["projector"]["clockwise"] = True
    return cfg


def rect_film_config(regular):
    cfg = benchy_index_matched(N=24, angles=16, regular_sampling=regular, spp=1 if regular else 2)
    cfg["sensor"]["film"] = {"type": "vfilm", "resx": 20, "resy": 30, "resz": 16}
    cfg["sensor"]["scalex"], cfg["sensor"]["scaley"], cfg["sensor"]["scalez"] = 8.0, 12.0, 6.0
    return cfg


def check(oracle, cfg, seed=3):
    d = desc_from_config(cfg)
    spp = 1 if cfg["regular_sampling"] else cfg["spp"]
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(seed)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    proj = Projection(d, DEV)
    got = proj.forward(torch.as_tensor(pat, device=DEV), None, spp, seed).cpu().numpy()[..., 0]
    ref, visits = oracle.forward(d, pat, spp=spp, seed=seed, nthreads=8)
    assert np.abs(ref).max() > 0
    assert rel_l2(got, ref) < RTOL
    assert abs(proj.count_visits(spp, seed) - visits) <= max(2, 1e-4 * visits)
    G = rng.uniform(-1, 1, got.shape).astype(np.float32)
    g = proj.adjoint(torch.as_tensor(G, device=DEV), n, None, spp, seed).cpu().numpy()
    gref, _ = oracle.adjoint(d, G, spp=spp, seed=seed, nthreads=8)
    assert rel_l2(g, gref) < RTOL
    proj.close()
    return d, got


@pytest.mark.parametrize("regular", [True, False])
def test_projector_crop(oracle, regular):
    d, dose = check(oracle, crop_config(regular))
    assert (d.crop_x, d.crop_y, d.crop_offset_x, d.crop_offset_y) == (4, 4, 8, 3)
    # test_projector.py:38: every ray of the crop has |o.z| < 2 -> no dose in slices beyond |z| = 2
    h = (d.bbox_max[2] - d.bbox_min[2]) / d.film_res[2]
    zc = d.bbox_min[2] + (0.5 + np.arange(d.film_res[2])) * h
    outside = np.abs(zc) > 2.0 + 0.5 * h
    assert outside.any() and np.all(dose[outside] == 0.0)
    assert dose[~outside].sum() > 0


@pytest.mark.parametrize("regular", [True, False])
def test_clockwise_motion(oracle, regular):
    cfg = clockwise_config(regular)
    d, dose = check(oracle, cfg)
    assert d.clockwise == 1
    # the clockwise render is the counter-clockwise one mirrored in y (x -> x, y -> -y) only for a
    # symmetric pattern set; here: it differs from the counter-clockwise render
    ccw = copy.deepcopy(cfg)
    ccw["projector"]["clockwise"] = False
    d2 = desc_from_config(ccw)
    n = d2.n_patterns * d2.crop_y * d2.crop_x
    pat = np.random.default_rng(3).uniform(0.0, 0.1, n).astype(np.float32)
    spp = 1 if regular else cfg["spp"]
    other = Projection(d2, DEV).forward(torch.as_tensor(pat, device=DEV), None, spp, 3).cpu().numpy()[..., 0]
    assert rel_l2(dose, other) > 1e-2


@pytest.mark.parametrize("regular", [True, False])
def test_rectangular_film(oracle, regular):
    d, dose = check(oracle, rect_film_config(regular))
    # film.py:9-11: res.x = props['resy'] (30), res.y = props['resx'] (20)
    assert tuple(d.film_res) == (30, 20, 16)
    assert dose.shape == (16, 20, 30)


@pytest.mark.parametrize("regular", [True, False])
def test_render_forward_is_the_jvp(oracle, regular):
    """render_forward (volume.py:58-95): the dose tangent of a pattern tangent.  The render is
    linear, so it equals the oracle's forward of the tangent, and a central difference of render
    along the tangent."""
    from drtvam_amd.integrators import VolumeIntegrator
    from drtvam_amd.optimize import load_scene
    from drtvam_amd.scene import load_dict
    cfg = benchy_index_matched(N=24, angles=12, regular_sampling=regular, spp=1 if regular else 2)
    cfg["projector"]["device"] = DEV
    scene = load_dict(load_scene(copy.deepcopy(cfg)))
    sensor = scene.sensor_by_id("sensor")
    integ = VolumeIntegrator({"regular_sampling": regular, "max_depth": 6, "rr_depth": 6})
    p = scene.projector
    n = p.active_size()
    rng = np.random.default_rng(7)
    base = torch.as_tensor(rng.uniform(0, 0.1, n).astype(np.float32), device=DEV)
    tan = torch.as_tensor(rng.uniform(-1, 1, n).astype(np.float32), device=DEV)
    spp = 1 if regular else 2
    p.active_data = base.clone().requires_grad_(True)
    p.active_data.grad = tan.clone()
    jvp = integ.render_forward(scene, None, sensor, seed=4, spp=spp).clone()
    ref, _ = oracle.forward(integ.desc(scene, sensor), tan.cpu().numpy(), spp=spp, seed=4, nthreads=8)
    assert rel_l2(jvp.cpu().numpy()[..., 0], ref) < RTOL
    eps = 1e-2
    with torch.no_grad():
        p.active_data = base + eps * tan
        hi = integ.render(scene, sensor, seed=4, spp=spp).clone().double()
        p.active_data = base - eps * tan
        lo = integ.render(scene, sensor, seed=4, spp=spp).clone().double()
    fd = (hi - lo) / (2 * eps)
    assert float(torch.linalg.norm(fd - jvp.double()) / torch.linalg.norm(jvp.double())) < 1e-4
    with pytest.raises(ValueError, match="tangent"):
        p.active_data = base.clone()
        integ.render_forward(scene, None, sensor)
