"""Oracle for the Radon filter (filter_radon; integrators/radon.py:47-106, optimize.py:143-163).

Known answers: a ray through a target box inside an index-matched vial carries
L = e^{-st t_in} (1 - e^{-st (t_out - t_in)}) (t counted from the ray origin, radon.py:95-98);
rays that miss the target carry 0; behind a glass vial the value picks up the Fresnel weight.
"""
import os

import numpy as np
import pytest

from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config
from drtvam_amd.utils import read_ply

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def box_tris():
    v, f = read_ply(os.path.join(GOLDEN, "occlusion.ply"))  # box x in [-1, 1], y in [-0.5, 0.5], z in [-0.25, 0.25]
    return np.asarray(v, np.float32)[np.asarray(f)]


def test_axial_ray_known_answer(oracle):
    d = desc_from_config(benchy_index_matched(N=21, angles=4, size_mm=5.0, r=2.9, regular_sampling=True))
    rad = oracle.radon(d, box_tris(), spp=1)
    W = 21
    wr = d.pixel_size_x * d.pixel_size_y * d.print_time
    st = d.sigma_t
    # angle 0, middle row (z = 0), middle column (y = 0): origin x = 20 - 0.005, runs along -x
    t_in = (20.0 - 0.005) - 1.0
    L = np.exp(-st * t_in) * (1 - np.exp(-st * 2.0))
    assert rad[10 * W + 10] == pytest.approx(wr * L, rel=1e-4)
    # a row above the box (z = 2.5 - 0.5 * 5/21 ... > 0.25) misses it
    assert rad[0 * W + 10] == 0.0


def test_support_is_the_target_shadow(oracle):
    d = desc_from_config(benchy_index_matched(N=24, angles=6, size_mm=5.0, r=2.9, regular_sampling=True))
    rad = oracle.radon(d, box_tris(), spp=1).reshape(6, 24, 24)
    pix = d.pixel_size_x
    for a in range(6):
        alpha = 2 * np.pi * a / 6
        c, s = np.cos(alpha), np.sin(alpha)
        for row in range(24):
            z = (0.5 - (row + 0.5) / 24) * 24 * pix
            for col in range(24):
                xc = (0.5 - (col + 0.5) / 24) * 24 * pix  # lateral offset: points (s, -c) * xc on the line
                # the line {(s, -c) xc + t (-c, -s)} meets the box iff its lateral distance fits the box
                hits = abs(z) < 0.25 and _line_hits_box(xc, c, s)
                if abs(abs(z) - 0.25) < 1e-3 or _near_edge(xc, c, s):
                    continue
                assert (rad[a, row, col] > 0) == hits, (a, row, col)


def _line_hits_box(xc, c, s):
    # project the box corners on the lateral axis (s, -c)
    corners = [(x, y) for x in (-1, 1) for y in (-0.5, 0.5)]
    lat = [x * s - y * c for x, y in corners]
    return min(lat) < xc < max(lat)


def _near_edge(xc, c, s):
    corners = [(x, y) for x in (-1, 1) for y in (-0.5, 0.5)]
    lat = [x * s - y * c for x, y in corners]
    return min(abs(xc - min(lat)), abs(xc - max(lat))) < 1e-3


def test_glass_vial_weights(oracle):
    d = desc_from_config(cylindrical_refraction(N=21, angles=2, size_mm=5.0, r_int=3.5, r_ext=4.0))
    rad = oracle.radon(d, box_tris(), spp=1)
    r = oracle.ray(d, 10 * 21 + 10)
    assert rad[10 * 21 + 10] > 0
    # axial ray: normal incidence on both interfaces; the value carries their weight
    wr = d.pixel_size_x * d.pixel_size_y * d.print_time
    L = rad[10 * 21 + 10] / wr
    t_in = (20.0 - 0.005) - 1.0
    assert L == pytest.approx(r["weight"] * np.exp(-d.sigma_t * t_in) * (1 - np.exp(-2 * d.sigma_t)), rel=1e-3)


def test_jittered_samples_and_threads(oracle):
    d = desc_from_config(benchy_index_matched(N=16, angles=5, size_mm=5.0, r=2.9, regular_sampling=False, spp=4))
    a = oracle.radon(d, box_tris(), spp=4, seed=3, nthreads=1)
    b = oracle.radon(d, box_tris(), spp=4, seed=3, nthreads=8)
    np.testing.assert_array_equal(a, b)
    assert (a > 0).sum() > 0 and (a == 0).sum() > 0
