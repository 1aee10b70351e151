"""GPU: compacted active sets (filter_radon / filter_nonzero, optimize.py:143-163,
projector.py:66-68) seed their sampler streams by position in the whole
projector.active_pixels (common.py:57-67 sampler.seed(seed, active_size * spp), :81
dr.repeat) and weight rays by the whole set's size (projector.py:164-165, :187).

* a sparse jittered set vs the oracle (which follows the same definition);
* the same set split over two angle-shard plans (desc.active_base / active_total): the
  shard doses sum to the unsharded dose and the shard gradients concatenate to the
  unsharded gradient, i.e. sharding draws exactly the reference's samples;
* TvamProblem under filter_radon optimises over the compacted set (L-BFGS vectors of the
  active size) and the optimised dose matches the dense masked run.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd.configs import benchy_index_matched, desc_from_config
from drtvam_amd.engine import Projection

RTOL_L2 = 1e-4


def rel_l2(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _desc(N, A, angle_range=None, **kw):
    return desc_from_config(benchy_index_matched(N=N, angles=A, **kw), angle_range=angle_range)


def _set(n, seed):
    rng = np.random.default_rng(seed)
    keep = np.sort(rng.choice(n, n // 3, replace=False)).astype(np.uint32)
    pat = rng.uniform(0.01, 0.1, keep.size).astype(np.float32)
    return keep, pat


def _t(a, dtype=None):
    return torch.as_tensor(a if dtype is None else a.astype(dtype), device="cuda:0").contiguous()


@pytest.mark.parametrize("spp", [1, 3])
def test_sparse_jittered_vs_oracle(oracle, spp):
    N, A = 24, 12
    d = _desc(N, A, regular_sampling=False, spp=spp)
    d.active_base, d.active_total = 1000, 0  # a later shard's streams
    n = A * N * N
    keep, pat = _set(n, 5)
    ref, _ = oracle.forward(d, pat, active_pixels=keep, spp=spp, seed=7)
    proj = Projection(d, "cuda:0")
    got = proj.forward(_t(pat), _t(keep, np.int32), spp, 7).cpu().numpy()[..., 0]
    assert rel_l2(got, ref) < RTOL_L2
    G = np.random.default_rng(6).uniform(-1, 1, (N, N, N)).astype(np.float32)
    gref, _ = oracle.adjoint(d, G, active_pixels=keep, spp=spp, seed=9)
    g = proj.adjoint(_t(G), keep.size, _t(keep, np.int32), spp, 9).cpu().numpy()
    assert rel_l2(g, gref) < RTOL_L2


def test_sparse_records_reused_and_dropped():
    """A sparse jittered set's ray records are kept per (active_pixels, count, seed, spp): a second
    forward of the same seed with new values, an adjoint of the same seed and slice-range
    forwards reuse them; an in-place change of active_pixels drops them (the engine calls
    tvam_plan_set_active).  Every result equals a fresh plan's."""
    N, A, spp = 24, 12, 2
    d = _desc(N, A, regular_sampling=False, spp=spp)
    n = A * N * N
    keep, pat = _set(n, 8)
    pat2 = np.random.default_rng(9).uniform(0.01, 0.1, keep.size).astype(np.float32)
    G = _t(np.random.default_rng(10).uniform(-1, 1, (N, N, N)).astype(np.float32))
    pix = _t(keep, np.int32)
    proj = Projection(d, "cuda:0")

    def fresh_forward(p, px, seed):
        q = Projection(d, "cuda:0")
        out = q.forward(_t(p), px, spp, seed)
        q.close()
        return out

    a = proj.forward(_t(pat), pix, spp, 7)
    b = proj.forward(_t(pat2), pix, spp, 7)  # reused records, new values
    assert torch.equal(b, fresh_forward(pat2, pix, 7))
    g = proj.adjoint(G, keep.size, pix, spp, 7)
    q = Projection(d, "cuda:0")
    assert torch.equal(g, q.adjoint(G, keep.size, pix, spp, 7))
    q.close()
    zc = proj.fwd_chunk
    if zc > 0:  # slice ranges of one forward assemble the whole forward
        out = torch.zeros_like(a)
        for z0 in range(0, N, zc):
            proj.forward_slices(_t(pat), pix, spp, 7, z0, min(N, z0 + zc), out)
        assert torch.equal(out, a)
    # in-place change of the set: same pointer and count, other pixels
    keep2 = np.sort(np.random.default_rng(11).choice(n, keep.size, replace=False)).astype(np.int32)
    pix.copy_(_t(keep2))
    c = proj.forward(_t(pat), pix, spp, 7)
    assert torch.equal(c, fresh_forward(pat, pix, 7))
    assert not torch.equal(c, a)
    proj.close()


def test_sparse_records_dropped_for_a_new_set_at_a_freed_address():
    """set A is used, then set B, then A is freed and set C (same count, other pixels)
    is allocated at A's old address.  A call on C with A's seed must not reuse A's ray records."""
    N, A, spp = 24, 12, 2
    d = _desc(N, A, regular_sampling=False, spp=spp)
    n = A * N * N
    keep_a, pat = _set(n, 8)
    keep_b = np.sort(np.random.default_rng(12).choice(n, keep_a.size, replace=False)).astype(np.int32)
    keep_c = np.sort(np.random.default_rng(13).choice(n, keep_a.size, replace=False)).astype(np.int32)
    proj = Projection(d, "cuda:0")
    pix_a = _t(keep_a, np.int32)
    addr = pix_a.data_ptr()
    proj.forward(_t(pat), pix_a, spp, 7)
    pix_b = _t(keep_b)
    proj.forward(_t(pat), pix_b, spp, 7)
    del pix_a
    torch.cuda.synchronize()
    pix_c = torch.empty(keep_c.size, dtype=torch.int32, device="cuda:0")  # the caching allocator's freed block
    pix_c.copy_(_t(keep_c))
    assert pix_c.data_ptr() == addr, "the allocator did not reuse the freed block (test premise)"
    got = proj.forward(_t(pat), pix_c, spp, 7)
    q = Projection(d, "cuda:0")
    assert torch.equal(got, q.forward(_t(pat), pix_c, spp, 7))
    q.close()
    proj.close()


@pytest.mark.parametrize("planar_regular", [False, True])
def test_sparse_set_split_over_angle_shards(planar_regular):
    """Two angle-shard plans over halves of one sparse set draw the unsharded set's samples."""
    N, A, spp = 24, 12, 2
    kw = dict(regular_sampling=planar_regular, spp=1 if planar_regular else spp)
    n = A * N * N
    keep, pat = _set(n, 8)
    full = Projection(_desc(N, A, **kw), "cuda:0")
    ref = full.forward(_t(pat), _t(keep, np.int32), spp, 3).cpu().numpy().astype(np.float64)
    G = np.random.default_rng(9).uniform(-1, 1, (N, N, N)).astype(np.float32)
    gref = full.adjoint(_t(G), keep.size, _t(keep, np.int32), spp, 4).cpu().numpy()
    cut = 5
    split = int(np.searchsorted(keep, cut * N * N))
    acc = np.zeros_like(ref)
    grads = []
    for (a0, a1), (i0, i1) in (((0, cut), (0, split)), ((cut, A), (split, keep.size))):
        part = Projection(_desc(N, A, angle_range=(a0, a1), **kw), "cuda:0")
        part.set_active(i0, keep.size)
        acc += part.forward(_t(pat[i0:i1]), _t(keep[i0:i1], np.int32), spp, 3).cpu().numpy()
        grads.append(part.adjoint(_t(G), i1 - i0, _t(keep[i0:i1], np.int32), spp, 4).cpu().numpy())
    assert rel_l2(acc, ref) < 1e-5
    assert rel_l2(np.concatenate(grads), gref) < 1e-5


def test_filter_radon_compacts_the_optimisation():
    """optimize.py:143-163: the active set after filter_radon holds only the pixels whose rays
    cross the target; the optimiser's vectors have that size and the patterns outside stay 0."""
    import copy
    import os
    from drtvam_amd.configs import BOX_HOLE_INDEX_MATCHED
    from drtvam_amd.optimize import TvamProblem
    cfg = copy.deepcopy(BOX_HOLE_INDEX_MATCHED)
    cfg["target"]["filename"] = os.path.join(os.path.dirname(__file__), "golden", "box_hole.ply")
    cfg["filter_radon"] = True
    cfg["spp_filter_radon"] = 2
    prob = TvamProblem(cfg, device=torch.device("cuda", 0))
    assert prob.active_pixels is not None
    assert 0 < prob.n_local < prob.n_global
    assert prob.x0.numel() == prob.n_local
    assert prob.proj.desc.active_total == prob.n_local
    losses = [prob.iteration(i) for i in range(6)]
    assert losses[-1] < losses[0]
    assert prob.patterns_local().numel() == prob.n_local
    dense = prob.gather_patterns(prob.patterns_local().float())
    assert dense.numel() == prob.n_global
    mask = torch.zeros(prob.n_global, dtype=torch.bool, device=dense.device)
    mask[prob.active_dense] = True
    assert float(dense[~mask].abs().max()) == 0.0
    # the compacted forward (jittered, 4 spp: streams by active position) vs the oracle
    from oracle import oracle
    pats = prob.patterns_local().float().contiguous()
    dose = prob.forward(pats, 3).cpu().numpy()[..., 0]
    d = prob.proj.desc.copy()
    ref, _ = oracle.forward(d, pats.cpu().numpy(), active_pixels=prob.active_pixels.cpu().numpy().astype(np.uint32),
                            spp=prob.spp, seed=3, nthreads=8)
    err = rel_l2(dose, ref)
    assert err < RTOL_L2, err

def test_filter_radon_analytic_target():
    """An analytic target (bench configs) filters by its bounding cuboid: rays above / below the
    occupied slices and beside its projection are dropped."""
    from drtvam_amd.optimize import TvamProblem
    cfg = benchy_index_matched(N=32, angles=8)
    cfg["filter_radon"] = True
    prob = TvamProblem(cfg, device=torch.device("cuda", 0))
    assert 0.3 * prob.n_global < prob.n_local < 0.9 * prob.n_global
    losses = [prob.iteration(i) for i in range(3)]
    assert losses[-1] < losses[0]
