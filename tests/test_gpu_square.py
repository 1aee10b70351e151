"""GPU parity for the square vial and occluder meshes (config 5).

Square vial: refracted rays (per-ray direction + weight records, chord-traced slot lists,
ray-driven planar forward / planar adjoint under regular sampling).  Occluders end the
medium segment at a z-dependent point, so those scenes run the per-ray tile kernels (each
ray's record carries its own segment end).  Same tolerance as the other parity tests.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config, square_vial
from drtvam_amd.engine import Projection
from parity_util import flip_protocol

OCC = os.path.join(os.path.dirname(__file__), "golden", "occlusion.ply")
RTOL = 1e-4


def rel_l2(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def make(N=24, A=12, vial="square", occ=False, regular=True, spp=1, planar=True, albedo=0.0, tile=0):
    occl = (OCC,) if occ else ()
    if vial == "square":
        cfg = square_vial(N=N, angles=A, regular_sampling=regular, spp=spp, occluders=occl)
    elif vial == "index_matched":
        cfg = benchy_index_matched(N=N, angles=A, size_mm=5.0, r=2.9, regular_sampling=regular, spp=spp)
        cfg["vial"]["occlusions"] = [{"filename": f} for f in occl]
    else:
        cfg = cylindrical_refraction(N=N, angles=A, size_mm=5.0, r_int=3.5, r_ext=4.0, regular_sampling=regular,
                                     spp=spp)
        cfg["vial"]["occlusions"] = [{"filename": f} for f in occl]
    if albedo:
        cfg["vial"]["medium"]["albedo"] = albedo
        cfg["vial"]["medium"]["phase"] = {"type": "rayleigh"}
    d = desc_from_config(cfg, tile=tile)
    if not planar:
        d.flags |= _abi.FLAG_NO_PLANAR
    return d


CASES = [
    dict(),                                   # square vial, planar adjoint + ray-driven forward
    dict(planar=False),
    dict(N=40, A=30, tile=7),
    dict(regular=False, spp=2),
    dict(occ=True),                           # occluder: per-ray tile kernels
    dict(occ=True, regular=False, spp=2),
    dict(vial="index_matched", occ=True),
    dict(vial="cylindrical", occ=True),
    dict(occ=True, albedo=0.9, N=20),         # box_hole_scattering-like: square vial, scattering, occluder
]


def _id(c):
    return "-".join(f"{k}{v}" for k, v in c.items()) or "default"


@pytest.mark.parametrize("case", CASES, ids=_id)
def test_forward_matches_oracle(oracle, case):
    spp = case.get("spp", 1)
    d = make(**case)
    n = d.n_patterns * d.crop_y * d.crop_x
    pat = np.random.default_rng(0).uniform(0.0, 0.1, n).astype(np.float32)
    ref, visits = oracle.forward(d, pat, spp=spp, seed=5, nthreads=8)
    assert np.max(ref) > 0
    proj = Projection(d, "cuda:0")
    got = proj.forward(torch.as_tensor(pat, device="cuda:0"), None, spp, 5).cpu().numpy()[..., 0]
    assert proj.planar == (case.get("regular", True) and case.get("planar", True) and not case.get("occ"))
    if case.get("albedo"):  # scattered paths: counted flips, 1e-4 on the rest (parity_util.py)
        G = np.random.default_rng(1).uniform(-1, 1, ref.shape).astype(np.float32)
        flip_protocol(oracle, proj, d, pat, G, spp, 5, nthreads=8)
    else:
        assert rel_l2(got, ref) < RTOL
    hv = proj.count_visits(spp, 5)
    assert abs(hv - visits) <= max(2, 1e-4 * visits)


@pytest.mark.parametrize("case", CASES, ids=_id)
def test_adjoint_matches_oracle(oracle, case):
    spp = case.get("spp", 1)
    d = make(**case)
    n = d.n_patterns * d.crop_y * d.crop_x
    G = np.random.default_rng(1).uniform(-1, 1, (d.film_res[2], d.film_res[1], d.film_res[0])).astype(np.float32)
    ref, _ = oracle.adjoint(d, G, spp=spp, seed=9, nthreads=8)
    proj = Projection(d, "cuda:0")
    g = proj.adjoint(torch.as_tensor(G, device="cuda:0"), n, None, spp, 9).cpu().numpy()
    if not case.get("albedo"):  # scattering: covered by the flip protocol of the forward test
        assert rel_l2(g, ref) < RTOL


@pytest.mark.parametrize("occ", [False, True])
def test_dot_product(occ):
    d = make(N=32, A=16, occ=occ, regular=False, spp=2)
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(2)
    p = torch.as_tensor(rng.uniform(0, 1, n).astype(np.float32), device="cuda:0")
    G = torch.as_tensor(rng.uniform(-1, 1, (32, 32, 32)).astype(np.float32), device="cuda:0")
    proj = Projection(d, "cuda:0")
    Ap = proj.forward(p, None, 2, 11)[..., 0]
    AtG = proj.adjoint(G, n, None, 2, 11)
    lhs = float(torch.sum(Ap.double() * G.double()))
    rhs = float(torch.dot(p.double(), AtG.double()))
    assert abs(lhs - rhs) <= 1e-5 * abs(lhs)
