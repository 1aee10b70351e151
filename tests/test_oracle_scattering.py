"""Oracle for scattering media (config 4).

The restated path loop (volume.py:179-272 with has_scattering) is pinned by:
  * phase-function moments (isotropic, Rayleigh (3/8)(1 + mu^2), Henyey-Greenstein <mu> = g)
    for planar and axis-aligned incident directions (coordinate_system() branches);
  * exact structure: first medium segment == (1 - albedo) x the non-scattering render, the
    parts sum to the whole, depth truncation, thread-count independence, the adjoint dot test;
  * an independent analog Monte Carlo (numpy RNG, rejection-sampled Rayleigh, collision
    tallies) of the scattered part, which has the same expectation as the reference's
    track-length estimator (analytic absorption along every segment up to the next surface).
Parity with Mitsuba's own sampler stream stays unpinned (no mitsuba here), as for jittered rays.
"""
import numpy as np
import pytest

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config


def scene(N=16, A=8, albedo=0.5, sigma_t=0.1, phase="rayleigh", vial="index_matched", max_depth=8, g=None,
          regular=True, spp=1, r=8.0):
    if vial == "index_matched":
        cfg = benchy_index_matched(N=N, angles=A, sigma_t=sigma_t, regular_sampling=regular, spp=spp, r=r)
    else:
        cfg = cylindrical_refraction(N=N, angles=A, sigma_t=sigma_t, regular_sampling=regular, spp=spp)
    cfg["vial"]["medium"]["albedo"] = albedo
    if albedo > 0:
        cfg["vial"]["medium"]["phase"] = {"type": phase} if g is None else {"type": phase, "g": g}
    cfg["max_depth"] = max_depth
    cfg["rr_depth"] = max_depth
    return desc_from_config(cfg)


def patterns(d, seed=0):
    n = d.n_patterns * d.crop_y * d.crop_x
    return np.random.default_rng(seed).uniform(0.0, 0.1, n).astype(np.float32)


DIRS = [(-1.0, 0.0, 0.0), (0.6, -0.8, 0.0), (0.0, 0.0, 1.0), (0.0, 0.0, -1.0), (0.48, 0.6, -0.64)]


@pytest.mark.parametrize("kind,g,m1,m2", [("isotropic", None, 0.0, 1 / 3), ("rayleigh", None, 0.0, 0.4),
                                          ("hg", 0.6, 0.6, None), ("hg", -0.3, -0.3, None)])
@pytest.mark.parametrize("dvec", DIRS)
def test_phase_moments(oracle, kind, g, m1, m2, dvec):
    d = scene(phase=kind, g=g)
    n = 96
    u = (np.arange(n) + 0.5) / n  # stratified grid
    dv = np.asarray(dvec, np.float32)
    mus = []
    for up in u:  # fine strata on the polar sample: u1 (rayleigh, hg), u2 for isotropic
        for ua in u[::4]:  # (square_to_uniform_sphere: z = 1 - 2 u.y, phi = 2 pi u.x)
            u1, u2 = (ua, up) if kind == "isotropic" else (up, ua)
            wo = oracle.phase(d, dv, u1, u2)
            assert abs(np.linalg.norm(wo) - 1.0) < 1e-5
            mus.append(float(np.dot(wo, dv)))
    mus = np.asarray(mus)
    assert abs(mus.mean() - m1) < 5e-3
    if m2 is not None:
        assert abs((mus ** 2).mean() - m2) < 5e-3


@pytest.mark.parametrize("vial", ["index_matched", "cylindrical"])
def test_first_segment_is_unscattered_render(oracle, vial):
    a = 0.4
    d = scene(albedo=a, vial=vial)
    d0 = scene(albedo=0.0, vial=vial)
    p = patterns(d)
    first, _ = oracle.forward(d, p, part=1, nthreads=4)
    ref, _ = oracle.forward(d0, p, nthreads=4)
    assert np.max(ref) > 0
    st = np.float64(d.sigma_t)
    sa_over_st = (st - np.float64(np.float32(d.albedo) * np.float32(d.sigma_t))) / st  # fp32 sigma_s (sensor.py:400)
    np.testing.assert_allclose(first, sa_over_st * ref, rtol=1e-9, atol=1e-15 * np.max(ref))


@pytest.mark.parametrize("vial", ["index_matched", "cylindrical"])
def test_parts_sum_and_threads(oracle, vial):
    d = scene(albedo=0.6, vial=vial, regular=False, spp=2)
    p = patterns(d)
    full1, v1 = oracle.forward(d, p, spp=2, seed=3, nthreads=1)
    full8, v8 = oracle.forward(d, p, spp=2, seed=3, nthreads=8)
    f1, _ = oracle.forward(d, p, spp=2, seed=3, part=1, nthreads=8)
    f0, _ = oracle.forward(d, p, spp=2, seed=3, part=0, nthreads=8)
    assert v1 == v8
    np.testing.assert_allclose(full8, full1, rtol=1e-10, atol=1e-14 * np.max(full1))
    np.testing.assert_allclose(f0 + f1, full1, rtol=1e-10, atol=1e-14 * np.max(full1))
    assert f0.sum() > 0.05 * f1.sum()  # scattering carries a visible share


def test_depth_truncation(oracle):
    # index matched: the first medium segment is path vertex 1; max_depth 2 ends the path after it
    d2 = scene(albedo=0.7, max_depth=2)
    d8 = scene(albedo=0.7, max_depth=8)
    p = patterns(d2)
    only, _ = oracle.forward(d2, p)
    first, _ = oracle.forward(d8, p, part=1)
    np.testing.assert_allclose(only, first, rtol=1e-12, atol=0)


def test_small_albedo_limit(oracle):
    d = scene(albedo=1e-5)
    d0 = scene(albedo=0.0)
    p = patterns(d)
    got, _ = oracle.forward(d, p)
    ref, _ = oracle.forward(d0, p)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 5e-5


@pytest.mark.parametrize("vial", ["index_matched", "cylindrical"])
def test_dot_product(oracle, vial):
    d = scene(albedo=0.5, vial=vial, regular=False, spp=2)
    p = patterns(d, 1)
    G = np.random.default_rng(2).uniform(-1, 1, (d.film_res[2], d.film_res[1], d.film_res[0])).astype(np.float32)
    Ap, _ = oracle.forward(d, p, spp=2, seed=7, nthreads=8)
    AtG, _ = oracle.adjoint(d, G, spp=2, seed=7, nthreads=8)
    lhs = float(np.sum(Ap * G.astype(np.float64)))
    rhs = float(np.dot(p.astype(np.float64), AtG))
    assert abs(lhs - rhs) <= 1e-5 * abs(lhs)  # the adjoint's delta_L = grad * inv_vol is fp32 (volume.py:130)


def _analog(d, oracle, photons, rng):
    """Analog Monte Carlo of the scattered part: from each ray's first medium segment,
    photons fly Exp(sigma_t) distances; collisions absorb with 1 - albedo or scatter
    (Rayleigh by rejection).  Tallies absorbed weight per voxel from the second segment on.
    Segments whose line leaves through the tube's open ends deposit nothing (si invalid)."""
    st, a = d.sigma_t, d.albedo
    r, half = d.vial_r, 0.5 * d.vial_height
    bmin, bmax = np.array(d.bbox_min, np.float64), np.array(d.bbox_max, np.float64)
    res = np.array(d.film_res)
    h = (bmax - bmin) / res
    tally = np.zeros(res[::-1], np.float64)
    A, H, W = d.n_patterns, d.res_y, d.res_x
    p0, v0, wt = [], [], []
    for ang in range(A):
        for row in range(H):
            for col in range(W):
                ry = oracle.ray(d, (ang * H + row) * W + col)
                if not ry["hit"]:
                    continue
                p0.append(ry["o2"])
                v0.append(ry["d2"])
                wt.append(ry["maxt"])
    p = np.repeat(np.asarray(p0, np.float64), photons, 0)
    v = np.repeat(np.asarray(v0, np.float64), photons, 0)
    L = np.repeat(np.asarray(wt, np.float64), photons, 0)
    alive = np.ones(len(p), bool)
    nseg = d.max_depth - 1  # index matched: medium segments at depths 1 .. max_depth - 1
    for seg in range(nseg):
        if seg > 0:  # distance to the tube wall from inside
            A2 = v[:, 0] ** 2 + v[:, 1] ** 2
            B = p[:, 0] * v[:, 0] + p[:, 1] * v[:, 1]
            C = p[:, 0] ** 2 + p[:, 1] ** 2 - r * r
            with np.errstate(divide="ignore", invalid="ignore"):
                L = (-B + np.sqrt(np.maximum(B * B - A2 * C, 0))) / A2
            zw = p[:, 2] + L * v[:, 2]
            alive &= (A2 > 0) & (np.abs(zw) <= half)
        s = rng.exponential(1.0 / st, len(p))
        coll = alive & (s < L)
        q = p + s[:, None] * v
        absorbed = coll & (rng.random(len(p)) >= a)
        if seg > 0:
            idx = np.floor((q - bmin) / h).astype(np.int64)
            inb = absorbed & np.all((idx >= 0) & (idx < res), axis=1)
            np.add.at(tally, (idx[inb, 2], idx[inb, 1], idx[inb, 0]), 1.0)
        scat = coll & ~absorbed
        # Rayleigh: mu with pdf (3/8)(1 + mu^2) by rejection; phi uniform; any basis around v
        mu = np.empty(len(p))
        todo = np.ones(len(p), bool)
        while todo.any():
            m = rng.uniform(-1, 1, todo.sum())
            ok = rng.uniform(0, 2, todo.sum()) < 1 + m * m
            sel = np.flatnonzero(todo)[ok]
            mu[sel] = m[ok]
            todo[sel] = False
        phi = rng.uniform(0, 2 * np.pi, len(p))
        ax = np.where(np.abs(v[:, 2:3]) < 0.9, np.array([[0, 0, 1.0]]), np.array([[1.0, 0, 0]]))
        e1 = np.cross(v, ax)
        e1 /= np.linalg.norm(e1, axis=1, keepdims=True)
        e2 = np.cross(v, e1)
        sn = np.sqrt(np.maximum(1 - mu * mu, 0))
        vn = mu[:, None] * v + (sn * np.cos(phi))[:, None] * e1 + (sn * np.sin(phi))[:, None] * e2
        p = np.where(scat[:, None], q, p)
        v = np.where(scat[:, None], vn, v)
        alive = scat
    return tally / photons


def test_scattered_part_matches_analog_mc(oracle):
    """E[scattered dose] of the oracle (16 seeds x 1 path per ray, jittered) vs analog MC."""
    d = scene(N=12, A=6, albedo=0.6, sigma_t=0.15, max_depth=6, r=5.0)
    n = d.n_patterns * d.crop_y * d.crop_x
    ones = np.ones(n, np.float32)
    # oracle scattered part with unit patterns, several seeds; weight -> per-ray energy units
    wr = (d.pixel_size_x * d.pixel_size_y * n / n) * d.print_time
    vol = np.prod((np.array(d.bbox_max) - np.array(d.bbox_min)) / np.array(d.film_res))
    tots, prof = [], []
    for seed in range(16):
        # regular sampling ignores the seed for the rays but the path loop draws from it
        f0, _ = oracle.forward(d, ones, seed=seed, part=0, nthreads=8)
        e = f0 * vol / wr / (1 - d.albedo)  # absorbed collisions per ray (analog units)
        tots.append(e.sum())
        prof.append(e.sum(axis=(1, 2)))
    tots = np.asarray(tots)
    analog = _analog(d, oracle, 400, np.random.default_rng(11))
    ta = analog.sum() / (1 - d.albedo)
    m, se = tots.mean(), tots.std(ddof=1) / np.sqrt(len(tots))
    assert m > 0
    assert abs(m - ta) < 4 * se + 0.01 * ta, (m, se, ta)
    # z profile (slices), coarse
    pz = np.mean(prof, axis=0)
    pa = analog.sum(axis=(1, 2)) / (1 - d.albedo)
    assert np.linalg.norm(pz - pa) / np.linalg.norm(pa) < 0.1


def test_subset_streams_match_whole_set(oracle):
    """oracle.forward / adjoint with `streams` (the subset entries' positions in the whole dense
    set) reproduce the whole set's per-pixel adjoint and, for patterns that vanish off the
    subset, its forward exactly: the checker of tests/test_gpu_bin_chunks.py."""
    d = scene(N=16, A=6, regular=False, spp=2, vial="cylindrical", max_depth=6)
    n = d.n_patterns * d.crop_y * d.crop_x
    sub = np.arange(3, n, 7)
    pix = np.arange(n, dtype=np.uint32)[sub]  # crop = the whole DMD here
    pat = np.zeros(n, np.float32)
    pat[sub] = np.random.default_rng(1).uniform(0.0, 0.1, sub.size)
    G = np.random.default_rng(2).uniform(-1, 1, (16, 16, 16)).astype(np.float32)
    d.active_total = n  # the subset's rays are weighted by the whole set's size
    whole, _ = oracle.forward(d, pat, spp=2, seed=9, nthreads=1)
    part, _ = oracle.forward(d, pat[sub], active_pixels=pix, spp=2, seed=9, nthreads=1, streams=sub)
    assert whole.sum() > 0
    np.testing.assert_allclose(part, whole, rtol=0, atol=1e-12 * np.abs(whole).max())
    gw, _ = oracle.adjoint(d, G, spp=2, seed=9, nthreads=2)
    gs, _ = oracle.adjoint(d, G, active_pixels=pix, spp=2, seed=9, nthreads=2, streams=sub)
    np.testing.assert_array_equal(gs, gw[sub])
    # without streams the subset would draw the streams of positions 0 .. |sub| - 1
    g0, _ = oracle.adjoint(d, G, active_pixels=pix, spp=2, seed=9, nthreads=2)
    assert not np.array_equal(g0, gw[sub])
