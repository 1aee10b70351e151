"""GPU parity for scattering media (config 4).

The GPU splits every path: the planar / tile kernels deposit its first medium
segment, `tvam_scatter_kernel` replays the sampler stream and runs the free
flights, phase sampling and 3-D DDA of the later segments.  The oracle runs
the whole path loop.  Both draw the same samples in the same order, so the
paths agree except where a last-ulp difference of logf / cbrtf / sincos (device
vs host libm) flips a comparison: the flip protocol of parity_util.py counts
those paths' pixels and holds the forward and adjoint of every other path to
1e-4 relative L2; the visit counts agree to 1e-4.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config
from drtvam_amd.engine import Projection
from parity_util import RTOL, flip_protocol


def rel_l2(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def make(N=24, A=12, vial="index_matched", albedo=0.5, sigma_t=0.1, phase="rayleigh", g=None, regular=True, spp=1,
         max_depth=8, rr_depth=None, planar=True):
    if vial == "index_matched":
        cfg = benchy_index_matched(N=N, angles=A, sigma_t=sigma_t, regular_sampling=regular, spp=spp)
    else:
        cfg = cylindrical_refraction(N=N, angles=A, sigma_t=sigma_t, regular_sampling=regular, spp=spp)
    cfg["vial"]["medium"]["albedo"] = albedo
    cfg["vial"]["medium"]["phase"] = {"type": phase} if g is None else {"type": phase, "g": g}
    cfg["max_depth"] = max_depth
    cfg["rr_depth"] = max_depth if rr_depth is None else rr_depth
    d = desc_from_config(cfg)
    if not planar:
        d.flags |= _abi.FLAG_NO_PLANAR
    return d


CASES = [
    dict(),                                             # index matched, planar first segments
    dict(planar=False),                                 # per-ray tile first segments
    dict(regular=False, spp=3),
    dict(vial="cylindrical"),
    dict(vial="cylindrical", regular=False, spp=2),
    dict(phase="isotropic", albedo=0.8, sigma_t=0.2),
    dict(phase="hg", g=0.7, N=20),
    dict(rr_depth=2, max_depth=12, albedo=0.9, sigma_t=0.3, N=16),  # Russian roulette after the 2nd segment
]


def _id(c):
    return "-".join(f"{k}{v}" for k, v in c.items()) or "default"


@pytest.mark.parametrize("case", CASES, ids=_id)
def test_matches_oracle(oracle, case):
    spp = case.get("spp", 1)
    d = make(**case)
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(0)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    G = rng.uniform(-1, 1, (d.film_res[2], d.film_res[1], d.film_res[0])).astype(np.float32)
    ref, visits = oracle.forward(d, pat, spp=spp, seed=5, nthreads=8)
    scat, _ = oracle.forward(d, pat, spp=spp, seed=5, nthreads=8, part=0)
    assert scat.sum() > 0.02 * ref.sum()  # the scattered part is exercised
    proj = Projection(d, "cuda:0")
    hv = proj.count_visits(spp, 5)
    assert abs(hv - visits) <= max(2, 1e-4 * visits)
    flip_protocol(oracle, proj, d, pat, G, spp, 5, nthreads=8)


@pytest.mark.parametrize("vial", ["index_matched", "cylindrical"])
def test_dot_product(vial):
    d = make(vial=vial, regular=False, spp=2, N=32, A=16)
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(2)
    p = torch.as_tensor(rng.uniform(0, 1, n).astype(np.float32), device="cuda:0")
    G = torch.as_tensor(rng.uniform(-1, 1, (32, 32, 32)).astype(np.float32), device="cuda:0")
    proj = Projection(d, "cuda:0")
    Ap = proj.forward(p, None, 2, 11)[..., 0]
    AtG = proj.adjoint(G, n, None, 2, 11)
    lhs = float(torch.sum(Ap.double() * G.double()))
    rhs = float(torch.dot(p.double(), AtG.double()))
    # <Ap, G> with G ~ U[-1, 1) cancels (|lhs| ~ 1e-2 of sum |Ap G|): fp32 per-path sums of the
    # adjoint and fp32 per-visit weights of the forward leave ~1e-7 of the terms, ~1e-5 of lhs
    scale = float(torch.sum((Ap.double() * G.double()).abs()))
    assert abs(lhs - rhs) <= 1e-6 * scale


def test_sparse_active_pixels(oracle):
    d = make(N=20, A=10)
    n = 10 * 20 * 20
    rng = np.random.default_rng(3)
    pat = rng.uniform(0.01, 0.1, n).astype(np.float32)
    keep = np.sort(rng.choice(n, n // 3, replace=False)).astype(np.uint32)
    ref, _ = oracle.forward(d, pat[keep], active_pixels=keep, seed=4)
    proj = Projection(d, "cuda:0")
    px = torch.as_tensor(keep.astype(np.int32), device="cuda:0")
    got = proj.forward(torch.as_tensor(pat[keep], device="cuda:0"), px, 1, 4).cpu().numpy()[..., 0]
    assert rel_l2(got, ref) < RTOL
    G = rng.uniform(-1, 1, (20, 20, 20)).astype(np.float32)
    gref, _ = oracle.adjoint(d, G, active_pixels=keep, seed=4)
    g = proj.adjoint(torch.as_tensor(G, device="cuda:0"), keep.size, px, 1, 4).cpu().numpy()
    assert rel_l2(g, gref) < RTOL


def test_seed_changes_scattering_only():
    """Regular sampling: the first segments are seed-independent, the scattered part is not."""
    d = make(N=20, A=10)
    n = 10 * 20 * 20
    p = torch.full((n,), 0.05, device="cuda:0")
    proj = Projection(d, "cuda:0")
    a = proj.forward(p, None, 1, 1)
    b = proj.forward(p, None, 1, 2)
    diff = float((a - b).abs().sum() / a.abs().sum())
    assert 1e-4 < diff < 0.5


def test_slab_refused():
    d = make(N=16, A=4)
    d.slab_begin, d.slab_end = 0, 8
    with pytest.raises(ValueError, match="slab"):
        Projection(d, "cuda:0")


@pytest.mark.parametrize("case", [dict(), dict(vial="cylindrical", regular=False, spp=2), dict(N=40, A=8, albedo=0.9)],
                         ids=_id)
def test_binned_matches_per_path(case):
    """Brick-binned scattered forward (LDS fixed point) and adjoint (LDS-staged gathers, per-entry
    partials) == the per-path global-atomic / global-gather kernels."""
    spp = case.get("spp", 1)
    d = make(**case)
    n = d.n_patterns * d.crop_y * d.crop_x
    p = torch.as_tensor(np.random.default_rng(4).uniform(0, 0.1, n).astype(np.float32), device="cuda:0")
    a = Projection(d, "cuda:0").forward(p, None, spp, 3)
    d2 = d.copy()
    d2.flags |= _abi.FLAG_SCATTER_ATOMIC
    b = Projection(d2, "cuda:0").forward(p, None, spp, 3)
    assert float(torch.linalg.norm(a - b) / torch.linalg.norm(b)) < 1e-5
    G = torch.as_tensor(np.random.default_rng(5).uniform(-1, 1, a.shape[:3]).astype(np.float32), device="cuda:0")
    ga = Projection(d, "cuda:0").adjoint(G, n, None, spp, 7)
    gb = Projection(d2, "cuda:0").adjoint(G, n, None, spp, 7)
    assert float(torch.linalg.norm(ga - gb) / torch.linalg.norm(gb)) < 1e-5


@pytest.mark.parametrize("chunk_slots", [None, "3000"], ids=["one-chunk", "many-chunks"])
def test_forward_bin_cache(monkeypatch, chunk_slots):
    """A second forward of the same seed reuses the cached brick bins (records rescaled to the new
    pattern): bit-identical to an uncached plan, for the cached seed, a new pattern and a new seed."""
    if chunk_slots:
        monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
        monkeypatch.setenv("TVAM_BIN_CHUNK_SLOTS", chunk_slots)
    import gc
    gc.collect()  # plans of earlier tests (their bin caches) and torch's cached blocks: the cache
    torch.cuda.empty_cache()  # stores a chunk only while a quarter of the device memory stays free
    d = make(vial="cylindrical", regular=False, spp=2, N=24, A=8)
    d.flags |= _abi.FLAG_NO_ZERO_SKIP  # the cache serves dense sets without zero skipping (as bench.py)
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(6)
    p1, p2 = (torch.as_tensor(rng.uniform(0, 0.1, n).astype(np.float32), device="cuda:0") for _ in range(2))
    cached = Projection(d, "cuda:0")
    got = [cached.forward(p1, None, 2, 3), cached.forward(p2, None, 2, 3), cached.forward(p1, None, 2, 3),
           cached.forward(p2, None, 2, 4)]
    st = cached.bin_stats()
    assert st["chunks"] >= (2 if chunk_slots else 1) and st["cached"] == 0 and st["stored"] == st["chunks"]
    # a cached call after the seed change: seed 4's records overwrote seed 3's in the same cache
    # buffers, and slots without a seed-4 segment must carry attenuation 0, not seed 3's
    got.append(cached.forward(p1, None, 2, 4))
    st = cached.bin_stats()
    assert st["cached"] == st["chunks"] >= 1, st
    print("bin stats", st)
    monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
    monkeypatch.setenv("TVAM_BIN_CACHE", "0")
    plain = Projection(d, "cuda:0")
    want = [plain.forward(p1, None, 2, 3), plain.forward(p2, None, 2, 3), plain.forward(p1, None, 2, 3),
            plain.forward(p2, None, 2, 4), plain.forward(p1, None, 2, 4)]
    assert plain.bin_stats()["cached"] == 0
    for a, b in zip(got, want):
        assert torch.equal(a, b)
    assert not torch.equal(got[1], got[3])
