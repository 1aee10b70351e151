"""CPU tests of the oracle (oracle/tvam_oracle.c): known answers and properties.

No reference test pins absolute dose values (mitsuba/drjit are not installed;
SURVEY.md section 8c), so the oracle is pinned by:
  * analytic known answers: a single axis-aligned ray's per-voxel
    exp(-s t_in) - exp(-s t_out) sums, and energy conservation of a full
    single-angle render (sum_v D V_vox = sum_rays w P (1 - e^{-s L}));
  * the reference's own property tests: crop bounds of
    tests/test_projector.py:7-38 and FD-vs-adjoint of
    tests/test_integrators.py:69-110 (< 2e-4 relative);
  * committed golden vectors (tests/golden/, made by tests/golden/make_golden.py)
    guarding against regressions of the restatement itself.
"""
import math
import os

import numpy as np
import pytest

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, desc_from_config

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def small_desc(N=16, A=8, **kw):
    cfg = benchy_index_matched(N=N, angles=A, **kw)
    return desc_from_config(cfg)


def test_single_ray_known_answer(oracle):
    # grid [-1,1]^3, 8^3 voxels; ray along +x through voxel row (y=3, z=5) centres
    d = _abi.default_desc()
    for a in range(3):
        d.bbox_min[a], d.bbox_max[a], d.film_res[a] = -1.0, 1.0, 8
    d.vial_r, d.sigma_t = 5.0, 0.7
    h = 0.25
    y, z = -1 + 3.5 * h, -1 + 5.5 * h
    o = np.array([-3.0, y, z], np.float32)
    film, visits = oracle.dda_ray(d, o, [1.0, 0.0, 0.0], 100.0, em=2.0)
    assert visits == 8
    expect = np.zeros((8, 8, 8))
    for i in range(8):
        t0, t1 = 2.0 + i * h, 2.0 + (i + 1) * h
        expect[5, 3, i] = 2.0 * (math.exp(-0.7 * t0) - math.exp(-0.7 * t1))
    np.testing.assert_allclose(film, expect, rtol=1e-6, atol=1e-12)


def test_single_ray_maxt_and_reverse(oracle):
    d = _abi.default_desc()
    for a in range(3):
        d.bbox_min[a], d.bbox_max[a], d.film_res[a] = -1.0, 1.0, 8
    d.vial_r, d.sigma_t = 5.0, 0.3
    h = 0.25
    o = np.array([3.0, -1 + 0.5 * h, -1 + 7.5 * h], np.float32)  # travelling -x, stops at t = 3.4
    film, visits = oracle.dda_ray(d, o, [-1.0, 0.0, 0.0], 3.4, em=1.0)
    # enters at x=1 (t=2), ends at x=-0.4 (t=3.4): voxels x=7..2 (last one partial)
    exp_vox = {7 - i: (2.0 + i * h, min(2.0 + (i + 1) * h, 3.4)) for i in range(6)}
    assert visits == 6
    for ix, (t0, t1) in exp_vox.items():
        assert film[7, 0, ix] == pytest.approx(math.exp(-0.3 * t0) - math.exp(-0.3 * t1), rel=1e-5)
    assert np.count_nonzero(film) == 6


def test_energy_single_angle(oracle):
    """One angle (alpha = 0, rays along -x): sum_v D V_vox equals the closed-form sum over rays."""
    N = 24
    d = small_desc(N=N, A=1)
    data = np.random.default_rng(0).uniform(0.0, 0.1, N * N).astype(np.float32)
    dose, visits = oracle.forward(d, data)
    h = 10.0 / N
    total = dose.sum() * h ** 3
    # closed form: ray (row, col) at y = -x_c, z = y_c, enters the grid at x = +5, leaves at x = -5;
    # its medium segment starts at the vial entry x = sqrt(r^2 - y^2) (spawn offset ~1e-4 ignored)
    r, s = d.vial_r, d.sigma_t
    ex = N * d.pixel_size_x
    w = d.pixel_size_x * d.pixel_size_y
    exp_total = 0.0
    for row in range(N):
        for col in range(N):
            xc = (0.5 - (col + 0.5) / N) * ex
            y = -xc
            xe = math.sqrt(r * r - y * y)
            t0, t1 = xe - 5.0, xe + 5.0
            exp_total += w * data[row * N + col] * (math.exp(-s * t0) - math.exp(-s * t1))
    assert total == pytest.approx(exp_total, rel=1e-4)
    assert visits == N * N * N  # every ray crosses N voxels


def test_crop_bounds(oracle):
    """tests/test_projector.py:7-38: 20x10 DMD, 4x4 crop at (8,3), distance 20 -> |o.y|, |o.z| < 2."""
    d = _abi.default_desc()
    d.n_patterns, d.res_x, d.res_y = 1, 20, 10
    d.crop_x = d.crop_y = 4
    d.crop_offset_x, d.crop_offset_y = 8, 3
    d.pixel_size_x = d.pixel_size_y = 1.0
    d.distance = 20.0
    d.vial_r = 5.0
    d.regular_sampling = 0
    for i in range(16):
        pixel = (3 + i // 4) * 20 + 8 + i % 4
        for k in range(128):
            r = oracle.ray(d, pixel, wave_index=i * 128 + k, seed=0)
            assert -2 < r["o"][1] < 2 and -2 < r["o"][2] < 2
            assert r["d"][0] == -1.0 and r["d"][1] == 0.0 and r["d"][2] == 0.0


def test_adjoint_dot_product(oracle):
    """<A p, G> == <p, A^T G> (the adjoint is the exact transpose of the forward)."""
    d = small_desc(N=16, A=12, regular_sampling=False, spp=2)
    n = 12 * 16 * 16
    rng = np.random.default_rng(1)
    p = rng.uniform(0, 1, n).astype(np.float32)
    G = rng.uniform(-1, 1, (16, 16, 16)).astype(np.float32)
    dose, _ = oracle.forward(d, p, spp=2, seed=3)
    g, _ = oracle.adjoint(d, G, spp=2, seed=3)
    lhs = float(np.sum(dose * G.astype(np.float64)))
    # the adjoint applies inv_vol in fp32 to G (volume.py:130), the forward in fp64
    rhs = float(np.dot(p.astype(np.float64), g))
    assert lhs == pytest.approx(rhs, rel=1e-6)


def test_fd_vs_adjoint(oracle):
    """tests/test_integrators.py:69-110 analogue: d mean(vol^2)/da by FD vs adjoint, < 2e-4 relative."""
    d = small_desc(N=16, A=16, regular_sampling=False, spp=2)
    n = 16 * 16 * 16
    pat = np.linspace(1, 10, n).astype(np.float32)
    eps = 1e-3
    v1, _ = oracle.forward(d, pat * (1 + eps), spp=2)
    v2, _ = oracle.forward(d, pat * (1 - eps), spp=2)
    fd = (np.mean(v1 ** 2) - np.mean(v2 ** 2)) / (2 * eps)
    v, _ = oracle.forward(d, pat, spp=2)
    G = (2 * v / v.size).astype(np.float32)
    g, _ = oracle.adjoint(d, G, spp=2)
    ad = float(np.dot(g, pat.astype(np.float64)))
    assert abs((ad - fd) / fd) < 2e-4


def test_parallel_equals_serial(oracle):
    d = small_desc(N=20, A=10)
    p = np.random.default_rng(2).uniform(0, 1, 10 * 20 * 20).astype(np.float32)
    a, va = oracle.forward(d, p, nthreads=1)
    b, vb = oracle.forward(d, p, nthreads=4)
    assert va == vb
    np.testing.assert_array_equal(a, b)


def test_sparse_active_set_matches_dense(oracle):
    d = small_desc(N=12, A=6)
    n = 6 * 144
    rng = np.random.default_rng(4)
    p = rng.uniform(0, 1, n).astype(np.float32)
    keep = np.nonzero(rng.uniform(size=n) > 0.5)[0].astype(np.uint32)
    dense = np.zeros(n, np.float32)
    dense[keep] = p[keep]
    a, _ = oracle.forward(d, dense)
    b, _ = oracle.forward(d, p[keep], active_pixels=keep)
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", ["im16_a8_regular", "im16_a8_jitter_spp2"])
def test_golden_vectors(oracle, name):
    """Regression guard of the restatement: committed vectors from tests/golden/make_golden.py."""
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    cfg = benchy_index_matched(N=int(z["N"]), angles=int(z["A"]), regular_sampling=bool(z["regular"]),
                               spp=int(z["spp"]))
    d = desc_from_config(cfg)
    dose, visits = oracle.forward(d, z["patterns"], spp=int(z["spp"]), seed=int(z["seed"]))
    assert visits == int(z["visits"])
    np.testing.assert_allclose(dose, z["dose"], rtol=1e-12, atol=1e-15)
    g, _ = oracle.adjoint(d, z["grad_dose"], spp=int(z["spp"]), seed=int(z["seed"]))
    np.testing.assert_allclose(g, z["grad"], rtol=1e-12, atol=1e-15)
