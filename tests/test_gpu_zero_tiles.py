"""GPU: the adjoints skip all-zero gradient tiles -- the list adjoint (tvam_adjl_kernel), the per-ray
tile adjoint (tvam_tile_kernel) and the brick-march adjoint of scattering media, whose all-zero
bricks write zero partials instead of marching.  The thresholded loss's gradient is exactly 0
wherever the dose meets its bounds, so whole (tile, slice chunk) / brick gradients are 0 in the
optimisation; here the gradient is 0 on the lower half of the slices (whole slice chunks, tiles and
bricks) and random above, and the adjoint still matches the oracle (which visits everything)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, desc_from_config
from drtvam_amd.engine import Projection
from parity_util import RTOL, flip_protocol, rel_l2


def half_zero_gradient(d, seed):
    """Random in [-1, 1] on the upper half of the slices, exactly 0 below."""
    G = np.random.default_rng(seed).uniform(-1, 1, (d.film_res[2], d.film_res[1], d.film_res[0])).astype(np.float32)
    G[: d.film_res[2] // 2] = 0.0
    return G


@pytest.mark.parametrize("planar,regular,spp", [(True, True, 1), (False, True, 1), (False, False, 2)],
                         ids=["list-adjoint", "tile-adjoint", "tile-adjoint-jittered"])
def test_zero_gradient_tiles_match_oracle(oracle, planar, regular, spp):
    N, A = 64, 24
    d = desc_from_config(benchy_index_matched(N=N, angles=A, regular_sampling=regular, spp=spp))
    if not planar:
        d.flags |= _abi.FLAG_NO_PLANAR
    n = d.n_patterns * d.crop_y * d.crop_x
    G = half_zero_gradient(d, 3)
    ref, _ = oracle.adjoint(d, G, spp=spp, seed=7, nthreads=8)
    proj = Projection(d, "cuda:0")
    try:
        assert proj.planar == planar
        g = proj.adjoint(torch.as_tensor(G, device="cuda:0"), n, None, spp, 7).cpu().numpy()
    finally:
        proj.close()
    assert np.abs(ref).max() > 0
    assert rel_l2(g, ref) < RTOL


def test_zero_gradient_bricks_match_oracle(oracle):
    """Scattering resin (32^3: two 32 x 32 x 16 bricks in z, the lower one's gradient all 0): the
    brick-march adjoint writes that brick's entries as zero partials; flip protocol vs the oracle."""
    cfg = benchy_index_matched(N=32, angles=12, sigma_t=0.1)
    cfg["vial"]["medium"]["albedo"] = 0.5
    cfg["vial"]["medium"]["phase"] = {"type": "rayleigh"}
    cfg["max_depth"] = cfg["rr_depth"] = 8
    d = desc_from_config(cfg)
    n = d.n_patterns * d.crop_y * d.crop_x
    pat = np.random.default_rng(0).uniform(0.0, 0.1, n).astype(np.float32)
    G = half_zero_gradient(d, 4)
    proj = Projection(d, "cuda:0")
    try:
        flip_protocol(oracle, proj, d, pat, G, 1, 5, nthreads=8)
    finally:
        proj.close()
