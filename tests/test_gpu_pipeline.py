"""GPU: the optimiser iteration in slab bands (lbfgs.DirectionPipeline, TvamProblem.direction_pipeline,
TvamProblem._iteration_pipelined, FusedLinearLBFGS.step_pipelined): band k's forward
(tvam_forward_slices), loss and adjoint (tvam_adjoint_slices: its DMD rows) on one stream while the
side stream runs the history pass (tvam_lbfgs_history_rows), the direction (tvam_lbfgs_direction_rows)
and the probes of the neighbouring bands.  It reproduces the unbanded optimisation: the same
per-element arithmetic, the loss / dots / probes summed over the bands (fp64 rounding only)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction
from drtvam_amd.optimize import TvamProblem


def _run(parts, N, steps=5, scene=benchy_index_matched):
    cfg = scene(N=N, angles=24)
    cfg["direction_parts"] = parts
    prob = TvamProblem(cfg, device=torch.device("cuda", 0))
    g = torch.Generator().manual_seed(1)
    prob.x0 = prob.local_from_global(torch.rand(prob.n_global, generator=g) * 0.1)
    for i in range(steps):
        prob.iteration(i)
    return prob, np.asarray(prob.loss_hist), prob.patterns_local().cpu().numpy()


@pytest.mark.parametrize("N,parts,scene", [(128, 2, benchy_index_matched), (192, 3, benchy_index_matched),
                                           (256, 3, benchy_index_matched), (128, 2, cylindrical_refraction)],
                         ids=["128-2", "192-3", "256-3", "cylindrical-128-2"])
def test_pipelined_direction_matches(N, parts, scene, monkeypatch):
    # band edges fall on multiples of the forward's and the adjoint's slice chunks: the default
    # 52-slice forward chunks leave these small films no common multiple, so the bands run at 32
    monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
    monkeypatch.setenv("TVAM_PLANAR_FWD_Z", "32")
    ref, loss0, x0 = _run(1, N, scene=scene)
    assert ref.opt.pipeline is None  # (the default: off)
    got, loss1, x1 = _run(parts, N, scene=scene)
    pipe = got.opt.pipeline
    assert pipe is not None and 2 <= len(pipe.parts) <= parts, pipe and pipe.parts
    # the bands tile the rows (in either order), the slice ranges the film
    bands = sorted((r0, r1) for r0, r1, _, _ in pipe.parts)
    assert bands[0][0] == 0 and bands[-1][1] == pipe.rows and all(a[1] == b[0] for a, b in zip(bands, bands[1:]))
    assert pipe.parts[0][2] == 0 and pipe.parts[-1][3] == got.proj.film_shape[0]
    assert all(a[3] == b[2] for a, b in zip(pipe.parts, pipe.parts[1:]))
    assert loss1[-1] < loss1[0]
    np.testing.assert_allclose(loss1, loss0, rtol=1e-6)
    np.testing.assert_allclose(x1, x0, rtol=1e-5, atol=1e-7)


def test_direction_rows_equal_full_direction():
    """tvam_lbfgs_direction_rows over bands that tile the rows == tvam_lbfgs_direction_dev (bit-identical)."""
    import ctypes
    from drtvam_amd import _abi
    lib = _abi.load_library()
    A, R, C, h = 7, 36, 44, 3
    n = A * R * C
    gen = torch.Generator().manual_seed(2)
    V = torch.randn(2 * h + 1, n, generator=gen).cuda()
    g, S, Y = V[0], [V[1 + j] for j in range(h)], [V[1 + h + j] for j in range(h)]
    coef = torch.randn(17, generator=gen).cuda()
    Sp = (ctypes.c_void_p * 8)(*[s.data_ptr() for s in S])
    Yp = (ctypes.c_void_p * 8)(*[y.data_ptr() for y in Y])
    st = torch.cuda.current_stream().cuda_stream
    full = torch.empty(n, device='cuda')
    _abi.check(lib.tvam_lbfgs_direction_dev(n, g.data_ptr(), h, Sp, Yp, coef.data_ptr(), full.data_ptr(), st))
    banded = torch.full((n,), float('nan'), device='cuda')
    for r0, r1 in ((0, 5), (5, 21), (21, 36)):
        _abi.check(lib.tvam_lbfgs_direction_rows(A, (r1 - r0) * C, R * C, r0 * C, g.data_ptr(), h, Sp, Yp,
                                                 coef.data_ptr(), banded.data_ptr(), st))
    assert torch.equal(full, banded)


@pytest.mark.parametrize("adjl_z", [None, "16"])
def test_adjoint_slices_assemble_the_adjoint(adjl_z, monkeypatch):
    """tvam_adjoint_slices over slab bands (rows from tvam_row_slices) == tvam_adjoint; also with the
    list adjoint's 16-slice workgroups on a film whose slab chunks are counted in 8-slice chunks
    (tvam_launch_adj_lists converts them)."""
    if adjl_z is not None:
        monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
        monkeypatch.setenv("TVAM_ADJL_Z", adjl_z)
    cfg = benchy_index_matched(N=128, angles=12)
    cfg["direction_parts"] = 2
    prob = TvamProblem(cfg, device=torch.device("cuda", 0))
    pipe = prob.direction_pipeline()
    assert pipe is not None
    gv = torch.rand(prob.proj.film_shape, device="cuda")
    full = prob.proj.adjoint(gv, prob.n_local)
    banded = torch.full((prob.n_local,), float("nan"), device="cuda")
    for r0, r1, z0, z1 in pipe.parts:
        prob.proj.adjoint_slices(gv, prob.n_local, z0, z1, r0, r1, banded)
    torch.testing.assert_close(banded, full, rtol=1e-6, atol=1e-6 * float(full.abs().max()))


def test_list_adjoint_matches_the_tile_adjoint(monkeypatch):
    """The list adjoint (visit lists built at plan creation, chunks claimed from an LDS counter,
    only groups holding chunks launched) against the per-ray tile adjoint on one plan's geometry
    (TVAM_ADJ_LISTS=0): the same weights in the same per-(ray, tile, slice) order, so equal to
    float-atomic ordering; on a full film and on an angle shard whose rays fill one step quadrant."""
    from drtvam_amd.configs import desc_from_config
    from drtvam_amd.engine import Projection
    N = 96
    for a0, a1 in [(0, N), (0, N // 8)]:
        d = desc_from_config(benchy_index_matched(N=N, angles=N))
        d.angle_begin, d.angle_end = a0, a1
        n = (a1 - a0) * int(d.crop_x) * int(d.crop_y)
        g = torch.rand((N, N, N), device="cuda", generator=torch.Generator(device="cuda").manual_seed(3)) - 0.5
        out = []
        for lists in ("1", "0"):
            monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
            monkeypatch.setenv("TVAM_ADJ_LISTS", lists)
            p = Projection(d, "cuda:0")
            try:
                assert p.planar
                out.append(p.adjoint(g, n, None, 1, 0))
            finally:
                p.close()
        torch.testing.assert_close(out[0], out[1], rtol=1e-5, atol=1e-6 * float(out[1].abs().max()))


def test_adjoint_lists_are_built_by_the_first_adjoint():
    """the planar adjoint's visit lists are built by a plan's first adjoint call, not at
    plan creation, so a forward-only plan (final_render) never allocates them; the adjoint's
    reported slice chunk is the same before and after the build, and the result is the oracle's
    (the list adjoint path of the other tests)."""
    from drtvam_amd.configs import desc_from_config
    from drtvam_amd.engine import Projection
    N = 160
    d = desc_from_config(benchy_index_matched(N=N, angles=N))
    n = N * int(d.crop_x) * int(d.crop_y)
    torch.cuda.synchronize()
    p = Projection(d, "cuda:0")
    try:
        chunk0 = p.adj_chunk
        x = torch.rand(n, device="cuda")
        p.forward(x, None, 1, 0)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        g = torch.rand((N, N, N), device="cuda")
        free_g = torch.cuda.mem_get_info()[0]
        p.adjoint(g, n, None, 1, 0)
        torch.cuda.synchronize()
        free1 = torch.cuda.mem_get_info()[0]
        lists = (free_g - free1) - n * 4  # device bytes the first adjoint added besides its output
        assert lists > 4 << 20, (free0, free_g, free1)
        assert p.adj_chunk == chunk0
    finally:
        p.close()
