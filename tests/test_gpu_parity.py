"""GPU parity tests: libtvam.so kernels vs the CPU oracle on identical inputs.

Tolerance (north star): forward dose within 1e-4 relative L2 of the reference
integrator; the kernels telescope exp() in fp32 and accumulate with LDS
atomics, the oracle accumulates in fp64, so the observed error is ~1e-6.
Visit counts and gradients are compared the same way.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, desc_from_config
from drtvam_amd.engine import Projection, render, loss_threshold

RTOL_L2 = 1e-4


def rel_l2(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def make(N, A, regular=True, spp=1, tile=0, angle_range=None, planar=True, zres=None, ray_fwd=False, xyres=None,
         **kw):
    """planar=False forces the per-ray tile kernels; zres != N gives 2 rows per slice
    (zres = N/2) or empty slices (zres = 2N); ray_fwd=True forces the ray-driven planar
    forward; xyres = N/4 makes the DMD 4x finer than the voxels (ray-driven forward)."""
    cfg = benchy_index_matched(N=N, angles=A, regular_sampling=regular, spp=spp, **kw)
    d = desc_from_config(cfg, angle_range=angle_range, tile=tile)
    if not planar:
        d.flags |= _abi.FLAG_NO_PLANAR
    if ray_fwd:
        d.flags |= _abi.FLAG_RAY_FWD
    if zres is not None:
        d.film_res[2] = zres
    if xyres is not None:
        d.film_res[0] = d.film_res[1] = xyres
    return d


def gpu_forward(desc, pat, spp=1, seed=0, pixels=None):
    proj = Projection(desc, "cuda:0")
    x = torch.as_tensor(pat, device="cuda:0").contiguous()
    px = None if pixels is None else torch.as_tensor(pixels.astype(np.int32), device="cuda:0")
    out = proj.forward(x, px, spp, seed)
    torch.cuda.synchronize()
    return out.cpu().numpy()[..., 0], proj


CASES = [
    dict(N=16, A=8),
    dict(N=32, A=24),
    dict(N=48, A=48, tile=16),          # many tile restarts
    dict(N=40, A=30, tile=7),           # ragged tiles
    dict(N=64, A=64),                   # config 1 (plumbing config, 64^3 / 64 angles)
    dict(N=32, A=16, regular=False, spp=3),
    dict(N=33, A=17, r=5.5),            # vial smaller than the grid's half-diagonal
    dict(N=32, A=24, planar=False),     # regular sampling on the per-ray tile kernels
    dict(N=40, A=30, tile=7, planar=False),
    dict(N=33, A=17, r=5.5, planar=False),
    dict(N=24, A=12, zres=12),          # two DMD rows per slice
    dict(N=24, A=12, zres=48),          # slices without rows
    dict(N=24, A=12, zres=12, planar=False),
    dict(N=32, A=24, ray_fwd=True),     # ray-driven planar forward
    dict(N=40, A=30, tile=7, ray_fwd=True),
    dict(N=24, A=12, zres=12, ray_fwd=True),
    dict(N=24, A=12, zres=48, ray_fwd=True),
    dict(N=64, A=16, xyres=16),         # DMD 4x finer than the voxels: ray-driven forward
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_forward_matches_oracle(oracle, case):
    case = dict(case)
    spp = case.get("spp", 1)
    d = make(**case)
    n = d.n_patterns * d.crop_y * d.crop_x
    pat = np.random.default_rng(0).uniform(0.0, 0.1, n).astype(np.float32)
    ref, visits = oracle.forward(d, pat, spp=spp, seed=5, nthreads=8)
    got, proj = gpu_forward(d, pat, spp=spp, seed=5)
    # planar path: regular sampling and every row's vial-entry offset row-independent (|z| <= 0.7 r)
    assert proj.planar == (case.get("regular", True) and case.get("planar", True) and 5.0 <= 0.7 * case.get("r", 8.0))
    assert proj.planar_forward == (proj.planar and not case.get("ray_fwd") and case.get("xyres") is None)
    assert rel_l2(got, ref) < RTOL_L2
    assert np.max(np.abs(got - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-7
    hv = proj.count_visits(spp, 5)
    assert abs(hv - visits) <= max(2, 1e-4 * visits)


@pytest.mark.parametrize("case", CASES[:5] + CASES[7:] + [dict(N=32, A=16, regular=False, spp=2)],
                         ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_adjoint_matches_oracle(oracle, case):
    case = dict(case)
    spp = case.get("spp", 1)
    d = make(**case)
    N = d.film_res[0]
    n = d.n_patterns * d.crop_y * d.crop_x
    G = np.random.default_rng(1).uniform(-1, 1, (d.film_res[2], d.film_res[1], N)).astype(np.float32)
    ref, _ = oracle.adjoint(d, G, spp=spp, seed=9, nthreads=8)
    proj = Projection(d, "cuda:0")
    g = proj.adjoint(torch.as_tensor(G, device="cuda:0"), n, None, spp, 9).cpu().numpy()
    assert rel_l2(g, ref) < RTOL_L2


@pytest.mark.parametrize("parts,split,fz,az,nt", [(1, 1, 32, 8, 1024), (3, 5, 28, 4, 512), (7, 2, 24, 16, 1024),
                                                   (2, 3, 8, 8, 256), (1, 2, 16, 4, 256)])
def test_work_splits_match_oracle(oracle, monkeypatch, parts, split, fz, az, nt):
    """Angle parts of the voxel-driven forward (partial doses summed in part order),
    ray-list splits of the planar adjoint, every forward slab depth Z, the adjoint's
    slices per workgroup and its workgroup size give the oracle's results (the plan
    picks them from the slab depth; forced here)."""
    monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
    monkeypatch.setenv("TVAM_FWD_PARTS", str(parts))
    monkeypatch.setenv("TVAM_ADJ_SPLIT", str(split))
    monkeypatch.setenv("TVAM_PLANAR_FWD_Z", str(fz))
    monkeypatch.setenv("TVAM_PLANAR_ADJ_Z", str(az))
    monkeypatch.setenv("TVAM_ADJ_NT", str(nt))
    d = make(N=40, A=30)
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(4)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    ref, _ = oracle.forward(d, pat, nthreads=8)
    got, proj = gpu_forward(d, pat)
    assert proj.planar_forward
    assert rel_l2(got, ref) < RTOL_L2
    G = rng.uniform(-1, 1, (40, 40, 40)).astype(np.float32)
    gref, _ = oracle.adjoint(d, G, nthreads=8)
    g = proj.adjoint(torch.as_tensor(G, device="cuda:0"), n, None, 1, 0).cpu().numpy()
    assert rel_l2(g, gref) < RTOL_L2


@pytest.mark.parametrize("case", [dict(N=40, A=30), dict(N=24, A=12, zres=12), dict(N=24, A=12, zres=48)],
                         ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_forward_direct_staging_matches_oracle(oracle, monkeypatch, case):
    """The voxel-driven forward staging its windows from the [row][col] patterns directly
    (TVAM_FWD_BIN=0) instead of the slice-binned copy: same results."""
    monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
    monkeypatch.setenv("TVAM_FWD_BIN", "0")
    d = make(**case)
    n = d.n_patterns * d.crop_y * d.crop_x
    pat = np.random.default_rng(6).uniform(0.0, 0.1, n).astype(np.float32)
    ref, _ = oracle.forward(d, pat, nthreads=8)
    got, proj = gpu_forward(d, pat)
    assert proj.planar_forward
    assert rel_l2(got, ref) < RTOL_L2


@pytest.mark.parametrize("regular", [False, True])
def test_dot_product_gpu(regular):
    d = make(N=48, A=40, regular=regular, spp=2)
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(2)
    p = torch.as_tensor(rng.uniform(0, 1, n).astype(np.float32), device="cuda:0")
    G = torch.as_tensor(rng.uniform(-1, 1, (48, 48, 48)).astype(np.float32), device="cuda:0")
    proj = Projection(d, "cuda:0")
    Ap = proj.forward(p, None, 2, 11)[..., 0]
    AtG = proj.adjoint(G, n, None, 2, 11)
    lhs = float(torch.sum(Ap.double() * G.double()))
    rhs = float(torch.dot(p.double(), AtG.double()))
    assert abs(lhs - rhs) <= 1e-5 * abs(lhs)


@pytest.mark.parametrize("planar", [True, False])
def test_sparse_active_pixels(oracle, planar):
    d = make(N=24, A=12, planar=planar)
    n = 12 * 24 * 24
    rng = np.random.default_rng(3)
    pat = rng.uniform(0.01, 0.1, n).astype(np.float32)
    keep = np.sort(rng.choice(n, n // 3, replace=False)).astype(np.uint32)
    # active_pixels are flat indices into the full DMD (here crop == full res)
    ref, _ = oracle.forward(d, pat[keep], active_pixels=keep)
    got, proj = gpu_forward(d, pat[keep], pixels=keep)
    assert rel_l2(got, ref) < RTOL_L2
    G = rng.uniform(-1, 1, (24, 24, 24)).astype(np.float32)
    gref, _ = oracle.adjoint(d, G, active_pixels=keep)
    g = proj.adjoint(torch.as_tensor(G, device="cuda:0"), keep.size,
                     torch.as_tensor(keep.astype(np.int32), device="cuda:0"), 1, 0).cpu().numpy()
    assert rel_l2(g, gref) < RTOL_L2


def test_angle_shards_sum_to_full():
    N, A = 32, 20
    full = make(N=N, A=A)
    n = A * N * N
    pat = np.random.default_rng(4).uniform(0, 0.1, n).astype(np.float32)
    ref, _ = gpu_forward(full, pat)
    acc = np.zeros_like(ref, dtype=np.float64)
    bounds = [0, 7, 13, 20]
    for a0, a1 in zip(bounds[:-1], bounds[1:]):
        d = make(N=N, A=A, angle_range=(a0, a1))
        part, _ = gpu_forward(d, pat[a0 * N * N:a1 * N * N])
        acc += part
    assert rel_l2(acc, ref) < 1e-5


def test_render_autograd_matches_adjoint():
    d = make(N=24, A=16)
    n = 16 * 24 * 24
    proj = Projection(d, "cuda:0")
    x = torch.rand(n, device="cuda:0", requires_grad=True)
    vol = render(proj, x, spp=1, seed=0)
    w = torch.rand_like(vol)
    (vol * w).sum().backward()
    g = proj.adjoint(w.contiguous(), n, None, 1, 0)
    torch.testing.assert_close(x.grad, g, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("K,reduction", [(1, "sum"), (2, "sum"), (2, "mean"), (3, "sum")])
def test_fused_loss_matches_torch(K, reduction):
    from drtvam_amd.loss import ThresholdedLoss
    lf = ThresholdedLoss({"K": K, "tl": 0.85, "tu": 0.95, "reduction": reduction, "weight_void": 1.3,
                          "weight_limit": 0.7})
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.rand((20, 30, 40, 1), generator=g) * 1.3).cuda()
    dx = (torch.rand((20, 30, 40, 1), generator=g) - 0.5).cuda()
    tgt = (torch.rand((20, 30, 40, 1), generator=g) > 0.5).float().cuda()
    pats = torch.zeros(10, device="cuda")
    xr = x.clone().requires_grad_(True)
    ref = lf(xr, tgt, pats)
    ref.backward()
    grad = torch.empty_like(x)
    v = lf.fused_value_grad(x, tgt, pats, grad)
    assert float(v) == pytest.approx(float(ref), rel=1e-5)
    torch.testing.assert_close(grad, xr.grad, rtol=1e-5, atol=1e-7)
    v2 = lf.fused_value(x, tgt, pats, dx, 0.37)
    assert float(v2) == pytest.approx(float(lf(x + 0.37 * dx, tgt, pats)), rel=1e-5)


@pytest.mark.parametrize("dist", ["signed", "heavy", "sparse_spikes"])
def test_forward_fixed_point_and_fallback(oracle, dist):
    """Signed (L-BFGS search direction) and heavy-tailed inputs: fixed-point and float-fallback tiles."""
    d = make(N=40, A=36, planar=False)
    d.flags |= _abi.FLAG_FWD_STATS
    n = 36 * 40 * 40
    rng = np.random.default_rng(7)
    if dist == "signed":
        pat = rng.uniform(-1, 1, n).astype(np.float32)
    elif dist == "heavy":
        pat = rng.standard_cauchy(n).astype(np.float32)
    else:
        pat = rng.uniform(0, 1e-3, n).astype(np.float32)
        pat[rng.choice(n, 5, replace=False)] = 1e4
    ref, _ = oracle.forward(d, pat)
    got, proj = gpu_forward(d, pat)
    fb = proj.fallback_tiles()
    assert rel_l2(got, ref) < RTOL_L2, fb
    if dist == "sparse_spikes":
        assert fb > 0  # a few outliers set the fixed-point step: those tiles take the float path
    elif dist == "signed":
        assert fb == 0


@pytest.mark.parametrize("planar", [True, False])
@pytest.mark.parametrize("band", [False, True])
def test_slab_plan_matches_full_film(planar, band):
    """A plan restricted to film slab [z0, z1) (and, like a z-slab rank, to the DMD rows
    feeding it) renders exactly those slices of the full forward, and its adjoint is the
    full adjoint of a gradient that vanishes outside the slab."""
    import ctypes
    N, A, z0, z1 = 32, 16, 9, 21
    d = make(N=N, A=A, planar=planar)
    n = A * N * N
    rng = np.random.default_rng(11)
    pat = rng.uniform(0, 0.1, n).astype(np.float32)
    full, proj = gpu_forward(d, pat)
    ds = d.copy()
    ds.slab_begin, ds.slab_end = z0, z1
    pats = pat
    r0, r1 = 0, N
    if band:
        m = np.empty(N, dtype=np.int32)
        _abi.check(_abi.load_library().tvam_row_slices(ctypes.byref(d), m.ctypes.data_as(ctypes.c_void_p)))
        rows = np.nonzero((m >= z0) & (m < z1))[0]
        r0, r1 = int(rows.min()), int(rows.max()) + 1
        ds.crop_offset_y, ds.crop_y = r0, r1 - r0
        pats = pat.reshape(A, N, N)[:, r0:r1, :].reshape(-1).copy()
    part, ps = gpu_forward(ds, pats)
    assert part.shape == (z1 - z0, N, N)
    assert ps.planar == planar
    np.testing.assert_allclose(part, full[z0:z1], rtol=1e-5, atol=1e-7 * np.abs(full).max())
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    Gz = np.zeros_like(G)
    Gz[z0:z1] = G[z0:z1]
    gfull = proj.adjoint(torch.as_tensor(Gz, device="cuda:0"), n, None, 1, 0).cpu().numpy()
    gs = ps.adjoint(torch.as_tensor(G[z0:z1].copy(), device="cuda:0"), pats.size, None, 1, 0).cpu().numpy()
    ref = gfull.reshape(A, N, N)[:, r0:r1, :].reshape(-1)
    assert rel_l2(gs, ref) < 1e-5


@pytest.mark.parametrize("Z", [40, 52])
def test_deep_slab_forward(oracle, monkeypatch, Z):
    """The deep-slab voxel-driven forward (Z = 40 / 52 slices per workgroup, binned staging; the
    plan picks 52 for the 50-slice slabs of 8 z-slab ranks) against the oracle, including a
    partial last chunk (60 slices)."""
    monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
    monkeypatch.setenv("TVAM_PLANAR_FWD_Z", str(Z))
    d = make(N=60, A=30)
    n = d.n_patterns * d.crop_y * d.crop_x
    pat = np.random.default_rng(11).uniform(0.0, 0.1, n).astype(np.float32)
    ref, _ = oracle.forward(d, pat, nthreads=8)
    got, proj = gpu_forward(d, pat)
    assert proj.planar_forward
    assert rel_l2(got, ref) < RTOL_L2


@pytest.mark.parametrize("kind", ["planar", "refracted", "tile_jittered", "square_occluder"])
def test_forward_slices_assemble_the_forward(kind):
    """tvam_forward_slices (the overlapped angle-shard all-reduce): slice ranges on the
    forward's chunks, rendered one after another into one buffer, give the whole forward."""
    from drtvam_amd.configs import cylindrical_refraction, square_vial
    if kind == "planar":
        d = make(N=48, A=24)
    elif kind == "refracted":
        d = desc_from_config(cylindrical_refraction(N=40, angles=20))
    elif kind == "tile_jittered":
        d = make(N=32, A=16, regular=False, spp=2)
    else:
        import os
        occ = os.path.join(os.path.dirname(__file__), "golden", "occlusion.ply")
        d = desc_from_config(square_vial(N=40, angles=16, spp=2, regular_sampling=False, occluders=(occ,)))
    proj = Projection(d, "cuda:0")
    zc = proj.fwd_chunk
    assert zc >= 1
    n = d.n_patterns * d.crop_y * d.crop_x
    x = torch.as_tensor(np.random.default_rng(12).uniform(0, 0.1, n).astype(np.float32), device="cuda:0")
    spp = 1 if d.regular_sampling else 2
    full = proj.forward(x, None, spp, 3).clone()
    out = torch.full_like(full, float("nan"))
    nz = full.shape[0]
    edges = sorted({0, nz} | {min(nz, zc * q) for q in (1, 3)})
    for z0, z1 in zip(edges[:-1], edges[1:]):
        proj.forward_slices(x, None, spp, 3, z0, z1, out)
    torch.cuda.synchronize()
    assert not torch.isnan(out).any()
    assert rel_l2(out.cpu().numpy(), full.cpu().numpy()) < 1e-6
    with pytest.raises(ValueError):
        proj.forward_slices(x, None, spp, 3, 0, nz + 1, out)


def test_forward_slices_unsupported_for_scattering():
    from drtvam_amd.configs import cylindrical_scattering
    d = desc_from_config(cylindrical_scattering(N=24, angles=8, spp=2))
    proj = Projection(d, "cuda:0")
    assert proj.fwd_chunk == 0
