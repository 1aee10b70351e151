"""Shared parity helpers (not a test module).

Monte Carlo paths (jittered sampling, scattering) draw the same samples in the same order on
the GPU and in the oracle, so each path is the same path on both sides.  A device-vs-host libm
difference in the last ulp (logf, cbrtf, sincosf) can still flip a comparison -- a free flight
ending one side of a surface, a Russian-roulette draw, a voxel boundary -- and send one path
elsewhere.  `flip_protocol` finds those paths' pixels from the per-pixel adjoint (same seed as
the forward: a flipped path changes its pixel's gradient macroscopically, every other pixel
agrees to fp32 rounding), counts them, and holds everything else to the north-star bar.
"""
import numpy as np
import torch

from parity_report import report

RTOL = 1e-4  # north star: 1e-4 relative L2


def rel_l2(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def flipped_pixels(g, gref, gabs, rtol=1e-3):
    """Pixels whose adjoint differs beyond fp32 rounding: |g - gref| > rtol * gabs, gabs = the oracle's
    adjoint of |G| (the pixel's sum of |terms|: a random-sign G lets a pixel's sum cancel far below
    its terms, so |gref| is no measure of the rounding a pixel can carry).  A flipped path moves
    its pixel by a sizeable part of one sample's share (1 / spp)."""
    g = np.asarray(g, np.float64)
    gref = np.asarray(gref, np.float64)
    return np.abs(g - gref) > rtol * np.asarray(gabs, np.float64) + 1e-12


def flip_protocol(oracle, proj, desc, pat, G, spp, seed, active_pixels=None, gpu_pixels=None, nthreads=16,
                  dev="cuda:0", max_flip_frac=1e-4):
    """Forward + adjoint parity at RTOL outside the flipped pixels.  Returns a dict of the
    measured numbers (flip count, errors) for the test to report.  `active_pixels`: the oracle's
    active set (of `desc`); `gpu_pixels`: the plan's (None: its dense shard)."""
    n = pat.size
    pix_t = None if gpu_pixels is None else torch.as_tensor(np.asarray(gpu_pixels).astype(np.int32), device=dev)
    g = proj.adjoint(torch.as_tensor(G, device=dev), n, pix_t, spp, seed).cpu().numpy()
    gref, _ = oracle.adjoint(desc, G, active_pixels=active_pixels, spp=spp, seed=seed, nthreads=nthreads)
    gabs, _ = oracle.adjoint(desc, np.abs(G), active_pixels=active_pixels, spp=spp, seed=seed, nthreads=nthreads)
    flip = flipped_pixels(g, gref, gabs)
    nflip = int(flip.sum())
    keep = ~flip
    e_adj = rel_l2(g[keep], gref[keep])
    # the forward over the same paths with the flipped pixels' patterns zeroed on both sides
    p2 = np.where(flip, 0.0, pat).astype(np.float32)
    got = proj.forward(torch.as_tensor(p2, device=dev), pix_t, spp, seed).cpu().numpy()[..., 0]
    ref, visits = oracle.forward(desc, p2, active_pixels=active_pixels, spp=spp, seed=seed, nthreads=nthreads)
    e_fwd = rel_l2(got, ref)
    out = {"pixels": int(n), "flipped": nflip, "rel_l2_adjoint": e_adj, "rel_l2_forward": e_fwd,
           "rel_l2_adjoint_all": rel_l2(g, gref), "visits": int(visits)}
    print("flip protocol:", out)
    report(flipped=nflip, of=int(n) * spp, rel_l2_adjoint=e_adj, rel_l2_forward=e_fwd)
    assert nflip <= max(2, max_flip_frac * n * spp), out  # flipped paths: at most 1e-4 of them
    assert e_adj < RTOL, out
    assert e_fwd < RTOL, out
    return out
