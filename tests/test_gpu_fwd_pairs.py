"""The voxel-driven planar forward with voxel pairs (TVAM_FWD_PX=2, opt-in: a thread owns two
neighbouring voxel columns of a 32 x 16 tile and reads each candidate slab once for both) against
the one-voxel variant (TVAM_FWD_PX=1) and the oracle.  Every voxel sums the same candidates in the
same order (the pair's extra union column misses the voxel: weight 0), so the doses are identical."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, desc_from_config
from drtvam_amd.engine import Projection
from parity_util import RTOL, rel_l2


def _plans(monkeypatch, d):
    monkeypatch.setenv("TVAM_FWD_PX", "1")
    one = Projection(d, "cuda:0")
    monkeypatch.setenv("TVAM_FWD_PX", "2")
    two = Projection(d, "cuda:0")
    assert one.planar_forward and two.planar_forward
    return one, two


@pytest.mark.parametrize("N,A,z", [(50, 24, 0), (64, 40, 16), (37, 19, 24), (96, 32, 32)])
def test_pairs_identical_to_single(oracle, monkeypatch, N, A, z):
    if z:
        monkeypatch.setenv("TVAM_PLANAR_FWD_Z", str(z))
    d = desc_from_config(benchy_index_matched(N=N, angles=A))
    d.flags |= _abi.FLAG_NO_ZERO_SKIP
    n = A * N * N
    pat = np.random.default_rng(N).uniform(0.0, 0.1, n).astype(np.float32)
    x = torch.as_tensor(pat, device="cuda:0")
    one, two = _plans(monkeypatch, d)
    d1 = one.forward(x, None, 1, 0)
    d2 = two.forward(x, None, 1, 0)
    assert torch.equal(d1, d2)
    ref, _ = oracle.forward(d, pat, nthreads=8)
    assert rel_l2(d2.cpu().numpy()[..., 0], ref) < RTOL
    # slice ranges of the forward (the angle-shard overlap) assemble the whole film
    zc = two.fwd_chunk
    assert zc > 0
    out = torch.zeros_like(d2)
    for z0 in range(0, N, zc):
        two.forward_slices(x, None, 1, 0, z0, min(N, z0 + zc), out)
    assert torch.equal(out, d2)


def test_pairs_on_a_slab_plan(monkeypatch):
    """A z-slab plan (slab sharding: the film's slices [z0, z1) and their DMD row band) with pairs
    equals the same slices of the full film (up to the order of the angle parts' partial sums)."""
    N, A = 48, 24
    cfg = benchy_index_matched(N=N, angles=A)
    full_d = desc_from_config(cfg)
    pat = np.random.default_rng(5).uniform(0.0, 0.1, A * N * N).astype(np.float32)
    x = torch.as_tensor(pat, device="cuda:0")
    monkeypatch.setenv("TVAM_FWD_PX", "2")
    full = Projection(full_d, "cuda:0").forward(x, None, 1, 0)
    from drtvam_amd.optimize import TvamProblem
    prob = TvamProblem(dict(cfg, shard="slab"), device=torch.device("cuda", 0), rank=1, world_size=3)
    xl = prob.local_from_global(torch.as_tensor(pat))
    part = prob.forward_local(xl, 0)
    assert rel_l2(part.cpu().numpy(), full[prob.z0:prob.z1].cpu().numpy()) < 1e-6
