"""Oracle for the 'ratio' and 'delta' sensors (sensor.py:112-295).

Known answers:
  * ratio tracking is unbiased for the DDA's analytic absorption: at a majorant mu the
    deposits of a segment have expected density mu * (st / mu) (1 - st / mu)^N(t) with N(t)
    Poisson(mu t), i.e. st e^{-st t}: over many sampler streams the ratio film converges to the
    DDA film of the same rays (regular sampling, non-scattering medium);
  * the delta (collision) estimator is unbiased for the same quantity in a scattering medium:
    its total over many streams matches the DDA render's total;
  * both are linear in the patterns for a fixed stream: exact adjoint dot tests;
  * delta on a purely absorbing medium is refused (volume.py:160-161).
"""
import numpy as np
import pytest

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config


def scene(sensor, albedo=0.0, regular=True, spp=1, N=12, A=6, sigma_t=0.4, majorant=2.0, vial="index_matched"):
    if vial == "index_matched":
        cfg = benchy_index_matched(N=N, angles=A, size_mm=4.0, r=2.9, sigma_t=sigma_t, regular_sampling=regular,
                                   spp=spp)
    else:
        cfg = cylindrical_refraction(N=N, angles=A, size_mm=4.0, r_int=3.5, r_ext=4.0, sigma_t=sigma_t,
                                     regular_sampling=regular, spp=spp)
    d = desc_from_config(cfg)
    d.albedo = albedo
    d.phase_type = _abi.PHASE_RAYLEIGH
    d.sensor_type = {"dda": _abi.SENSOR_DDA, "ratio": _abi.SENSOR_RATIO, "delta": _abi.SENSOR_DELTA}[sensor]
    d.majorant = majorant
    return d


def pats(d, seed=0):
    return np.random.default_rng(seed).uniform(0.0, 0.1, d.n_patterns * d.crop_y * d.crop_x).astype(np.float32)


@pytest.mark.parametrize("vial", ["index_matched", "cylindrical"])
def test_ratio_converges_to_dda(oracle, vial):
    dr = scene("ratio", vial=vial, majorant=8.0)
    dd = scene("dda", vial=vial)
    p = pats(dr)
    ref, _ = oracle.forward(dd, p, nthreads=8)
    acc = np.zeros_like(ref)
    S = 48
    for seed in range(S):
        f, _ = oracle.forward(dr, p, seed=seed, nthreads=8)
        acc += f
    acc /= S
    assert acc.sum() == pytest.approx(ref.sum(), rel=5e-3)
    # voxel-wise: the Poisson noise of S streams (~2.7 deposits per voxel crossing, ~6 crossings
    # per voxel and stream: ~4 % expected)
    assert np.linalg.norm(acc - ref) / np.linalg.norm(ref) < 0.08


def test_delta_matches_dda_in_scattering_medium(oracle):
    dl = scene("delta", albedo=0.6, regular=False, spp=2, sigma_t=0.5)
    dd = scene("dda", albedo=0.6, regular=False, spp=2, sigma_t=0.5)
    p = pats(dl)
    tot_d, tot_l = 0.0, 0.0
    for seed in range(24):
        tot_d += oracle.forward(dd, p, spp=2, seed=seed, nthreads=8)[0].sum()
        tot_l += oracle.forward(dl, p, spp=2, seed=seed, nthreads=8)[0].sum()
    assert tot_l == pytest.approx(tot_d, rel=0.02)


@pytest.mark.parametrize("sensor,albedo", [("ratio", 0.0), ("ratio", 0.5), ("delta", 0.5)])
def test_estimator_dot_product(oracle, sensor, albedo):
    d = scene(sensor, albedo=albedo, regular=False, spp=2)
    rng = np.random.default_rng(3)
    p = rng.uniform(0, 1, d.n_patterns * d.crop_y * d.crop_x).astype(np.float32)
    G = rng.uniform(-1, 1, (12, 12, 12)).astype(np.float32)
    Ap, _ = oracle.forward(d, p, spp=2, seed=7, nthreads=8)
    AtG, _ = oracle.adjoint(d, G, spp=2, seed=7, nthreads=8)
    lhs = float(np.sum(Ap * G.astype(np.float64)))
    rhs = float(np.dot(p.astype(np.float64), AtG))
    assert abs(Ap).max() > 0
    assert lhs == pytest.approx(rhs, rel=1e-6)


def test_threads_agree(oracle):
    d = scene("ratio", albedo=0.5, regular=False, spp=2)
    p = pats(d)
    a, va = oracle.forward(d, p, spp=2, seed=1, nthreads=1)
    b, vb = oracle.forward(d, p, spp=2, seed=1, nthreads=8)
    assert va == vb
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-18)


def test_delta_needs_scattering(oracle):
    d = scene("delta", albedo=0.0)
    with pytest.raises(ValueError):
        oracle.forward(d, pats(d))


# ---------------------------------------------------------------------------
# Surface-aware films (film_channels 2) with the ratio / delta sensors (sensor.py:148-151, :257-260)
# ---------------------------------------------------------------------------
def sa_scene(sensor, tris, **kw):
    d = scene(sensor, **kw)
    d.film_channels = 2
    d.set_target(tris)
    return d


def _box():
    from test_oracle_surface import cube_tris
    return cube_tris([-1.1, -0.7, -0.9], [0.8, 1.3, 0.6])


@pytest.mark.parametrize("sensor,albedo", [("ratio", 0.0), ("ratio", 0.6), ("delta", 0.6)])
def test_surface_estimator_target_never_hit_equals_one_channel(oracle, sensor, albedo):
    """A target no path reaches: every deposit goes to channel 1, exactly the one-channel film."""
    from test_oracle_surface import cube_tris
    kw = dict(albedo=albedo, regular=False, spp=2, majorant=3.0)
    d2 = sa_scene(sensor, cube_tris([-0.5, -0.5, 30.0], [0.5, 0.5, 31.0]), **kw)
    d1 = scene(sensor, **kw)
    N = d1.film_res[0]
    p = pats(d1)
    ones = np.ones((N, N, N, 2), np.float32)
    sa, v2 = oracle.forward_surface(d2, p, ones, spp=2, seed=4, nthreads=8)
    ref, v1 = oracle.forward(d1, p, spp=2, seed=4, nthreads=8)
    vv = float(np.prod((np.asarray(d1.bbox_max) - np.asarray(d1.bbox_min)) / N))
    assert v1 == v2 and ref.sum() > 0
    assert np.all(sa[..., 0] == 0)
    np.testing.assert_allclose(sa[..., 1] / vv, ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("sensor,albedo", [("ratio", 0.0), ("delta", 0.6)])
def test_surface_estimator_channels_follow_target_side(oracle, sensor, albedo):
    d = sa_scene(sensor, _box(), albedo=albedo, regular=False, spp=2, majorant=3.0, N=16, A=8)
    N = 16
    sa, _ = oracle.forward_surface(d, pats(d, 2), np.ones((N, N, N, 2), np.float32), spp=2, seed=7, nthreads=8)
    lo, hi = [-1.1, -0.7, -0.9], [0.8, 1.3, 0.6]
    h = 4.0 / N
    c = -2.0 + h * (np.arange(N) + 0.5)
    z, y, x = np.meshgrid(c, c, c, indexing="ij")
    deep_in = (x > lo[0] + h) & (x < hi[0] - h) & (y > lo[1] + h) & (y < hi[1] - h) & (z > lo[2] + h) & (z < hi[2] - h)
    far_out = (x < lo[0] - h) | (x > hi[0] + h) | (y < lo[1] - h) | (y > hi[1] + h) | (z < lo[2] - h) | (z > hi[2] + h)
    assert np.all(sa[..., 1][deep_in] == 0) and np.all(sa[..., 0][far_out] == 0)
    assert sa[..., 0].sum() > 0 and sa[..., 1].sum() > 0


def test_surface_ratio_converges_to_surface_dda(oracle):
    """Ratio tracking on a surface-aware film is unbiased for the DDA surface film, channel by
    channel (non-scattering medium, regular sampling: the DDA film is deterministic)."""
    kw = dict(regular=True, majorant=8.0, N=12, A=6)
    dr = sa_scene("ratio", _box(), **kw)
    dd = sa_scene("dda", _box(), **kw)
    N = 12
    ones = np.ones((N, N, N, 2), np.float32)
    p = pats(dr)
    ref, _ = oracle.forward_surface(dd, p, ones, nthreads=8)
    acc = np.zeros_like(ref)
    S = 48
    for seed in range(S):
        f, _ = oracle.forward_surface(dr, p, ones, seed=seed, nthreads=8)
        acc += f
    acc /= S
    for ch in (0, 1):
        assert acc[..., ch].sum() == pytest.approx(ref[..., ch].sum(), rel=1e-2)
    assert np.linalg.norm(acc - ref) / np.linalg.norm(ref) < 0.1


@pytest.mark.parametrize("sensor,albedo", [("ratio", 0.0), ("delta", 0.6)])
def test_surface_estimator_dot_product(oracle, sensor, albedo):
    d = sa_scene(sensor, _box(), albedo=albedo, regular=False, spp=2, majorant=3.0)
    N = d.film_res[0]
    vol = oracle.compute_volume(d, sample_count=32, nthreads=8)
    rng = np.random.default_rng(5)
    p = rng.uniform(0, 1, d.n_patterns * N * N).astype(np.float32)
    G = rng.uniform(-1, 1, (N, N, N, 2)).astype(np.float32)
    Ap, _ = oracle.forward_surface(d, p, vol, spp=2, seed=3, nthreads=8)
    AtG, _ = oracle.adjoint_surface(d, G, vol, spp=2, seed=3, nthreads=8)
    lhs = float(np.sum(Ap * G.astype(np.float64)))
    rhs = float(np.dot(p.astype(np.float64), AtG))
    assert lhs == pytest.approx(rhs, rel=1e-6)
