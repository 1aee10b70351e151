"""The planar adjoint's per-(tile, step quadrant) ray lists (TVAM_ADJ_QUAD=1, tvam_plan.hip
adj_quadrant_lists: row pitch +-1 mod 16 by quadrant, lanes dealt by entry LDS chunk, blocks sorted
by in-tile length) against the oracle and the default (angle, column)-ordered lists."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config
from drtvam_amd.engine import Projection
from parity_util import RTOL, rel_l2


@pytest.mark.parametrize("mk", [benchy_index_matched, cylindrical_refraction], ids=["index_matched", "cylindrical"])
@pytest.mark.parametrize("block", ["256", "64"])
def test_quadrant_lists_match(oracle, monkeypatch, mk, block):
    N, A = 60, 36
    d = desc_from_config(mk(N=N, angles=A))
    n = A * N * N
    G = np.random.default_rng(3).uniform(-1, 1, (N, N, N)).astype(np.float32)
    Gt = torch.as_tensor(G, device="cuda:0")
    plain = Projection(d, "cuda:0")
    assert plain.planar
    g0 = plain.adjoint(Gt, n, None, 1, 0).cpu().numpy()
    monkeypatch.setenv("TVAM_ADJ_QUAD", "1")
    monkeypatch.setenv("TVAM_ADJ_QBLOCK", block)
    quad = Projection(d, "cuda:0")
    g1 = quad.adjoint(Gt, n, None, 1, 0).cpu().numpy()
    ref, _ = oracle.adjoint(d, G, nthreads=8)
    assert rel_l2(g1, g0) < 1e-6  # every (ray, tile) once: the same sums up to the atomics' order
    assert rel_l2(g1, ref) < RTOL


@pytest.mark.parametrize("mk", [benchy_index_matched, cylindrical_refraction], ids=["index_matched", "cylindrical"])
@pytest.mark.parametrize("split", ["1", "3"])
def test_ray_pairs_match(oracle, monkeypatch, mk, split):
    """The opt-in ray pairs (TVAM_ADJ_PAIR=1, tvam_plan.hip adj_pair_lists: ray j with ray j + ceil(n / 2) of each
    angle's crossing rays, one lane) against the plain (angle, column) lists and the oracle, with
    the tile's list split over 1 and 3 workgroups (parts of whole pairs)."""
    N, A = 60, 36
    d = desc_from_config(mk(N=N, angles=A))
    n = A * N * N
    G = np.random.default_rng(4).uniform(-1, 1, (N, N, N)).astype(np.float32)
    Gt = torch.as_tensor(G, device="cuda:0")
    monkeypatch.setenv("TVAM_ADJ_SPLIT", split)
    monkeypatch.setenv("TVAM_ADJ_PAIR", "0")
    plain = Projection(d, "cuda:0")
    assert plain.planar
    g0 = plain.adjoint(Gt, n, None, 1, 0).cpu().numpy()
    monkeypatch.setenv("TVAM_ADJ_PAIR", "1")
    paired = Projection(d, "cuda:0")
    g1 = paired.adjoint(Gt, n, None, 1, 0).cpu().numpy()
    ref, _ = oracle.adjoint(d, G, nthreads=8)
    assert rel_l2(g1, g0) < 1e-6  # every (ray, tile) once: the same sums up to the atomics' order
    assert rel_l2(g1, ref) < RTOL
