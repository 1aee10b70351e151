"""BASELINE.json's GPU configs at their full size against the CPU oracle.

  * config 2 (index matched, 400^3, 400 angles, regular sampling): the whole forward and
    adjoint, every angle, at 1e-4 relative L2, and the exact visit count;
  * config 3 (cylindrical vial, 400^3, 400 angles): the whole 400-angle forward -- whose int32
    fixed-point scale comes from a bound over all angles and the beam compression behind the
    refracting vial -- must take the fixed-point path with headroom and match at 1e-4; the
    adjoint on a 3-angle shard;
  * config 4 (cylindrical vial, scattering resin, 16 jittered rays per pixel): one angle of the
    400-angle scene (160 K pixels, 2.56 M paths);
  * config 5 (square vial + occluder, 800^3, 4 jittered rays per pixel): one angle of the
    800-angle scene (640 K pixels, 2.56 M rays).
Configs 4-5 use the flip protocol of parity_util.py (flipped-path pixels counted, 1e-4 on the rest).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import (benchy_index_matched, cylindrical_refraction, cylindrical_scattering,
                                desc_from_config, square_occluded)
from drtvam_amd.engine import Projection
from parity_report import report
from parity_util import RTOL, flip_protocol, rel_l2

DEV = "cuda:0"
THREADS = 16


def test_config2_every_angle(oracle):
    N = 400
    d = desc_from_config(benchy_index_matched(N=N, angles=N))
    n = N * N * N
    rng = np.random.default_rng(0)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    proj = Projection(d, DEV)
    assert proj.planar_forward
    got = proj.forward(torch.as_tensor(pat, device=DEV), None, 1, 0).cpu().numpy()[..., 0]
    ref, visits = oracle.forward(d, pat, nthreads=THREADS)
    e = rel_l2(got, ref)
    report(rel_l2_forward=e, visits=int(visits))
    print(f"config 2 forward rel-L2 {e:.3e}, visits {visits}")
    assert e < RTOL
    assert abs(proj.count_visits(1, 0) - visits) <= max(2, 1e-4 * visits)
    del got, ref
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    g = proj.adjoint(torch.as_tensor(G, device=DEV), n, None, 1, 0).cpu().numpy()
    gref, _ = oracle.adjoint(d, G, nthreads=THREADS)
    e = rel_l2(g, gref)
    report(rel_l2_adjoint=e)
    print(f"config 2 adjoint rel-L2 {e:.3e}")
    assert e < RTOL
    proj.close()


def test_config3_full_forward_fixed_point(oracle):
    """Both planar forwards of config 3 against one oracle run: the voxel-driven one (per-(tile,
    angle) chord-index models) and the ray-driven one, whose int32 fixed-point scale rests on a
    beam-compression bound over all 400 angles."""
    N = 400
    d = desc_from_config(cylindrical_refraction(N=N, angles=N))
    n = N * N * N
    pat = np.random.default_rng(1).uniform(0.0, 0.1, n).astype(np.float32)
    proj = Projection(d, DEV)
    assert proj.planar and proj.planar_forward  # the voxel-driven forward over refracted chords
    vox = proj.forward(torch.as_tensor(pat, device=DEV), None, 1, 0).cpu().numpy()[..., 0]
    proj.close()
    d.flags |= _abi.FLAG_RAY_FWD
    proj = Projection(d, DEV)
    assert proj.planar and not proj.planar_forward  # the ray-driven planar forward
    got = proj.forward(torch.as_tensor(pat, device=DEV), None, 1, 0).cpu().numpy()[..., 0]
    scale, fixed = proj.fwd_scale()
    assert fixed, "config 3 fell back to float LDS adds"
    ref, visits = oracle.forward(d, pat, nthreads=THREADS)
    # the largest fixed-point voxel sum the kernel formed (dose = sum * inv_vol / scale)
    h = [(d.bbox_max[a] - d.bbox_min[a]) / d.film_res[a] for a in range(3)]
    inv_vol = 1.0 / (h[0] * h[1] * h[2])
    peak = float(np.abs(ref).max()) / inv_vol * scale
    ev = rel_l2(vox, ref)
    print(f"config 3 voxel-driven forward rel-L2 {ev:.3e}")
    assert ev < RTOL
    e = rel_l2(got, ref)
    print(f"config 3 forward rel-L2 {e:.3e}, fixed-point scale 2^{np.log2(scale):.0f}, "
          f"largest sum {peak:.3e} of 2^31 ({peak / 2.0 ** 31:.3f}), visits {visits}")
    assert peak < 2.0 ** 30  # the guarantee of tvam_fwd_scale_kernel holds at full size
    assert peak > 2.0 ** 20  # ... and leaves >= 20 bits of the int32 to the largest sum
    assert e < RTOL
    assert abs(proj.count_visits(1, 0) - visits) <= max(2, 1e-4 * visits)
    proj.close()


def test_config3_adjoint_angle_shard(oracle):
    N, a0, a1 = 400, 137, 140
    d = desc_from_config(cylindrical_refraction(N=N, angles=N), angle_range=(a0, a1))
    dfull = desc_from_config(cylindrical_refraction(N=N, angles=N))
    n = (a1 - a0) * N * N
    rng = np.random.default_rng(2)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    pix = (a0 * N * N + np.arange(n)).astype(np.uint32)
    proj = Projection(d, DEV)
    got = proj.forward(torch.as_tensor(pat, device=DEV), None, 1, 0).cpu().numpy()[..., 0]
    assert proj.planar_forward
    ref, _ = oracle.forward(dfull, pat, active_pixels=pix, nthreads=THREADS)
    assert rel_l2(got, ref) < RTOL
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    g = proj.adjoint(torch.as_tensor(G, device=DEV), n, None, 1, 0).cpu().numpy()
    gref, _ = oracle.adjoint(dfull, G, active_pixels=pix, nthreads=THREADS)
    e = rel_l2(g, gref)
    report(rel_l2_adjoint=e)
    print(f"config 3 shard adjoint rel-L2 {e:.3e}")
    assert e < RTOL
    proj.close()


def _one_angle(oracle, cfg, N, a0, spp, seed):
    d = desc_from_config(cfg, angle_range=(a0, a0 + 1))
    dfull = desc_from_config(cfg)
    n = N * N
    # the shard is entries [a0 n, a0 n + n) of the whole dense set: the oracle's sparse call
    # draws the streams of those positions, and both weight rays by the whole set's size
    dfull.active_base = a0 * n
    d.active_total = dfull.active_total = N * n
    rng = np.random.default_rng(seed)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    pix = (a0 * N * N + np.arange(n)).astype(np.uint32)
    proj = Projection(d, DEV)
    out = flip_protocol(oracle, proj, dfull, pat, G, spp, seed, active_pixels=pix, nthreads=THREADS)
    proj.close()
    return out


def test_config4_one_angle_16spp(oracle):
    N = 400
    out = _one_angle(oracle, cylindrical_scattering(N=N, angles=N), N, 137, 16, 3)
    assert out["pixels"] == N * N


def test_config5_one_angle_800(oracle):
    N = 800
    out = _one_angle(oracle, square_occluded(N=N, angles=N), N, 291, 4, 4)
    assert out["pixels"] == N * N
