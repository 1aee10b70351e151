"""The production brick-bin path of config 4 against the oracle.

`bench.py --config 4` renders the scattered segments of its 1.02 G paths in chunks of 128 M
segment slots (23 chunks), each with its own int fixed-point scale from the chunk's largest
|weight|, and the line-search forward of an iteration reuses the cached records of the first
forward, reweighted to the new pattern (tvam_scatter.hip `tvam_scatter_binned`,
`tvam_bin_reweight_kernel`).  These tests run that path on the full 400^3, 16-spp scene:

  (i)   a 20-angle shard, which the default chunking splits into >= 2 chunks;
  (ii)  the same shard with TVAM_BIN_CHUNK_SLOTS forced down to >= 8 chunks (forward and adjoint);
  (iii) a second forward of the same seed with a new pattern: every chunk served from the cache;
  (iv)  all 400 angles (23 chunks), as the bench runs them;

and config 5 (800^3, square vial + occluder, 4 spp) on a 4-angle shard.

The GPU renders the whole dense shard.  The oracle traces a fixed subset of its pixels (every
53rd) with the shard's own sampler streams (`oracle.forward(..., streams=)`, the pixels' dense
positions): the forward's patterns are nonzero only on that subset, so the GPU's dose over the
whole shard is the oracle's dose of the subset, and the adjoint is compared on the subset.  The
flip protocol of parity_util.py (flipped-path pixels counted, then zeroed on both sides) holds
the rest to 1e-4 relative L2.  Reference: integrators/volume.py:179-272, sensor.py:306-440.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import cylindrical_scattering, desc_from_config, square_occluded
from drtvam_amd.engine import Projection
from parity_report import report
from parity_util import RTOL, flip_protocol, flipped_pixels, rel_l2

DEV = "cuda:0"
THREADS = 16
N4, A0, NA, SPP4, SEED4, STRIDE = 400, 120, 20, 16, 3, 53


def _make_shard(oracle, a0, na, stride):
    """Config 4's angles [a0, a0 + na): the subset's oracle adjoints / forwards, its flipped pixels
    and the GPU plan with the adjoint of the whole shard done."""
    cfg = cylindrical_scattering(N=N4, angles=N4)
    per = N4 * N4  # crop = the whole 400 x 400 DMD
    d = desc_from_config(cfg, angle_range=(a0, a0 + na))
    d.flags |= _abi.FLAG_NO_ZERO_SKIP  # as bench.py: every path marched, so the bin cache is used
    dfull = desc_from_config(cfg)
    d.active_total = dfull.active_total = N4 * per
    n = na * per
    sub = np.arange(0, n, stride, dtype=np.int64)
    pix = (a0 * per + sub).astype(np.uint32)     # full-DMD pixel index of each subset entry
    pos = (a0 * per + sub).astype(np.uint64)     # ... and its position in the dense set (its streams)
    rng = np.random.default_rng(7)
    G = rng.uniform(-1, 1, (N4, N4, N4)).astype(np.float32)
    gref, _ = oracle.adjoint(dfull, G, active_pixels=pix, spp=SPP4, seed=SEED4, nthreads=THREADS, streams=pos)
    gabs, _ = oracle.adjoint(dfull, np.abs(G), active_pixels=pix, spp=SPP4, seed=SEED4, nthreads=THREADS, streams=pos)
    proj = Projection(d, DEV)
    g = proj.adjoint(torch.as_tensor(G, device=DEV), n, None, SPP4, SEED4).cpu().numpy()[sub]
    # flip threshold 1e-4 of the pixel's sum of |terms| (flip_protocol: 1e-3): over 20 angles a
    # few paths flip in a late, low-weight segment and move their pixel by 2e-4 .. 9e-4 of it,
    # while fp32 rounding leaves < 1e-5 at the 99th percentile (tools/diag_chunks.py,
    # profiles/r03/diag_chunks.log); _check_adjoint asserts that rounding level on the rest
    flip = flipped_pixels(g, gref, gabs, rtol=1e-4)
    pats = []
    for k in range(2):  # two patterns on the subset (flipped pixels zeroed)
        p = np.where(flip, 0.0, rng.uniform(0.0, 0.1, sub.size)).astype(np.float32)
        ref, visits = oracle.forward(dfull, p, active_pixels=pix, spp=SPP4, seed=SEED4, nthreads=THREADS, streams=pos)
        pats.append((p, ref))
    return dict(d=d, n=n, sub=sub, G=G, gref=gref, gabs=gabs, flip=flip, g_default=g, pats=pats, proj=proj)


@pytest.fixture(scope="module")
def shard4(oracle):
    s = _make_shard(oracle, A0, NA, STRIDE)
    yield s
    s["proj"].close()
    torch.cuda.empty_cache()


@pytest.fixture
def full4(oracle):
    """All 400 angles of config 4 (the bench's 1.02 G paths, 23 chunks), every 50th pixel checked."""
    s = _make_shard(oracle, 0, N4, 50)
    yield s
    s["proj"].close()
    torch.cuda.empty_cache()


def _dense(s, p):
    full = np.zeros(s["n"], np.float32)
    full[s["sub"]] = p
    return torch.as_tensor(full, device=DEV)


def _check_adjoint(s, g):
    keep = ~s["flip"]
    nflip = int(s["flip"].sum())
    e = rel_l2(g[keep], s["gref"][keep])
    r99 = float(np.quantile(np.abs(g - s["gref"])[keep] / s["gabs"][keep], 0.99))
    report(flipped=nflip, of=int(s["sub"].size) * SPP4, rel_l2_adjoint=e, p99=r99)
    print(f"adjoint: {s['sub'].size} subset pixels, {nflip} flipped, rel-L2 {e:.3e}, "
          f"99th percentile |g - ref| / sum|terms| {r99:.2e}")
    assert nflip <= max(2, 1e-4 * s["sub"].size * SPP4)
    assert r99 < 1e-5
    assert e < RTOL


def _default_chunks(s, min_chunks):
    proj = s["proj"]
    st = proj.bin_stats()  # of the fixture's adjoint
    assert st["chunks"] >= min_chunks and st["count_mismatch"] == 0, st
    _check_adjoint(s, s["g_default"])
    (p1, ref1), (p2, ref2) = s["pats"]
    got = proj.forward(_dense(s, p1), None, SPP4, SEED4).cpu().numpy()[..., 0]
    st = proj.bin_stats()
    print("forward bin stats", st)
    # chunks are cached while an eighth of the device memory stays free: the rest (if any) run
    # uncached again in the second forward, next to the cached ones
    assert st["chunks"] >= min_chunks and st["cached"] == 0 and st["stored"] >= 1, st
    assert st["count_mismatch"] == 0, st  # the fill's walks agree with the writer's closed-form counts
    stored = st["stored"]
    e1 = rel_l2(got, ref1)
    got = proj.forward(_dense(s, p2), None, SPP4, SEED4).cpu().numpy()[..., 0]
    st = proj.bin_stats()
    print("cached forward bin stats", st)
    assert st["chunks"] >= min_chunks and st["cached"] == stored, st
    e2 = rel_l2(got, ref2)
    print(f"config 4 shard, {st['chunks']} chunks: forward rel-L2 {e1:.3e}, cached forward {e2:.3e}")
    assert e1 < RTOL and e2 < RTOL


def test_config4_shard_default_chunks(shard4):
    """(i) + (iii): the default 128 M-slot chunking of a 20-angle shard (>= 2 chunks), then the
    cached second forward of the same seed with a new pattern."""
    _default_chunks(shard4, 2)


def test_config4_all_angles(full4):
    """The bench's whole config-4 pass: 400 angles in 23 default chunks, adjoint, forward and the
    cached forward of the same seed; 1 pixel in 50 (25.6 K per angle's 160 K ... 1.28 M pixels,
    20.5 M paths) traced by the oracle."""
    _default_chunks(full4, 23)


def test_config4_shard_many_chunks(shard4, monkeypatch):
    """(ii): the same shard in >= 8 chunks (forward, cached forward and adjoint)."""
    s, proj = shard4, shard4["proj"]
    monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
    monkeypatch.setenv("TVAM_BIN_CHUNK_SLOTS", str(1 << 24))
    (p1, ref1), (p2, ref2) = s["pats"]
    got = proj.forward(_dense(s, p1), None, SPP4, SEED4).cpu().numpy()[..., 0]
    st = proj.bin_stats()
    assert st["chunks"] >= 8 and st["cached"] == 0 and st["stored"] >= 1 and st["count_mismatch"] == 0, st
    stored = st["stored"]
    e1 = rel_l2(got, ref1)
    got = proj.forward(_dense(s, p2), None, SPP4, SEED4).cpu().numpy()[..., 0]
    st = proj.bin_stats()
    assert st["chunks"] >= 8 and st["cached"] == stored, st
    e2 = rel_l2(got, ref2)
    print(f"config 4 shard, {st['chunks']} chunks: forward rel-L2 {e1:.3e}, cached forward {e2:.3e}")
    assert e1 < RTOL and e2 < RTOL
    g = proj.adjoint(torch.as_tensor(s["G"], device=DEV), s["n"], None, SPP4, SEED4).cpu().numpy()[s["sub"]]
    st = proj.bin_stats()
    assert st["chunks"] >= 8 and st["count_mismatch"] == 0, st
    _check_adjoint(s, g)


def test_config5_four_angle_shard(oracle):
    """Config 5 (800^3, 800 angles, 4 spp, square vial + occluder) on angles [291, 295)."""
    N, a0, na, spp, seed = 800, 291, 4, 4, 4
    cfg = square_occluded(N=N, angles=N)
    d = desc_from_config(cfg, angle_range=(a0, a0 + na))
    dfull = desc_from_config(cfg)
    per = N * N
    n = na * per
    dfull.active_base = a0 * per
    d.active_total = dfull.active_total = N * per
    rng = np.random.default_rng(seed)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    pix = (a0 * per + np.arange(n)).astype(np.uint32)
    proj = Projection(d, DEV)
    out = flip_protocol(oracle, proj, dfull, pat, G, spp, seed, active_pixels=pix, nthreads=THREADS)
    proj.close()
    assert out["pixels"] == n


def test_config5_spread_angles(oracle):
    """Config 5 (800^3, 800 angles, 4 spp, square vial + occluder) rendered whole on the GPU; the
    oracle traces 32 angles spread over the 800 (every 25th), every 16th pixel of each, with the
    whole set's sampler streams.  Forward: patterns nonzero on that subset only; adjoint: compared
    on the subset.  Flip protocol as above (flipped pixels counted and zeroed)."""
    N, spp, seed = 800, 4, 4
    cfg = square_occluded(N=N, angles=N)
    d = desc_from_config(cfg)
    dfull = desc_from_config(cfg)
    per = N * N
    n = N * per
    d.active_total = dfull.active_total = n
    angles = np.arange(0, N, 25)
    assert angles.size == 32
    sub = np.concatenate([a * per + np.arange(0, per, 16, dtype=np.int64) for a in angles])
    pix = sub.astype(np.uint32)
    pos = sub.astype(np.uint64)
    rng = np.random.default_rng(seed)
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    gref, _ = oracle.adjoint(dfull, G, active_pixels=pix, spp=spp, seed=seed, nthreads=THREADS, streams=pos)
    gabs, _ = oracle.adjoint(dfull, np.abs(G), active_pixels=pix, spp=spp, seed=seed, nthreads=THREADS, streams=pos)
    proj = Projection(d, DEV)
    try:
        g = proj.adjoint(torch.as_tensor(G, device=DEV), n, None, spp, seed).cpu().numpy()[sub]
        flip = flipped_pixels(g, gref, gabs)
        nflip = int(flip.sum())
        keep = ~flip
        ea = rel_l2(g[keep], gref[keep])
        p = np.where(flip, 0.0, rng.uniform(0.0, 0.1, sub.size)).astype(np.float32)
        ref, _ = oracle.forward(dfull, p, active_pixels=pix, spp=spp, seed=seed, nthreads=THREADS, streams=pos)
        full = np.zeros(n, np.float32)
        full[sub] = p
        got = proj.forward(torch.as_tensor(full, device=DEV), None, spp, seed).cpu().numpy()[..., 0]
        ef = rel_l2(got, ref)
        ts = proj.tile_stats()  # the tile kernels' stray rays (tvam_plan_tile_stats)
    finally:
        proj.close()
        torch.cuda.empty_cache()
    report(flipped=nflip, of=int(sub.size) * spp, rel_l2_adjoint=ea, rel_l2_forward=ef, strays=ts["strays"])
    print(f"config 5, 32 angles spread over 800, {sub.size} subset pixels ({sub.size * spp} paths): "
          f"{nflip} flipped, adjoint rel-L2 {ea:.3e}, forward rel-L2 {ef:.3e}; tile stats {ts}")
    # stray lists in use, each (tile, slice) workgroup walking its slice's strays: a tiny share of
    # the main-row slots on config 5 (its rows meet slice boundaries only at the extreme jitters)
    assert ts["spp"] == spp and 0 <= ts["strays"] <= ts["stray_cap"]
    assert ts["stray_walk"] == ts["strays"] * ts["tiles"]
    assert ts["main_walk"] > 0 and ts["stray_walk"] < 1e-3 * ts["main_walk"]
    assert nflip <= max(2, 1e-4 * sub.size * spp)
    assert ea < RTOL and ef < RTOL
