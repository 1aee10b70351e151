"""GPU: the fused L-BFGS step (tvam_lbfgs_history / _direction / tvam_axpy_clamp)
against the torch LinearLBFGS restatement of lbfgs.py:146-275 on a linear
least-squares problem (same render_fn / loss / Armijo)."""
import numpy as np
import pytest
import torch

from drtvam_amd.lbfgs import FusedLinearLBFGS, LinearLBFGS

pytestmark = pytest.mark.gpu


def _problem(n, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    A = (torch.randn(k, n, generator=g) / n ** 0.5).cuda()
    b = torch.randn(k, generator=g).cuda()
    return A, b


@pytest.mark.parametrize("n,clamp", [(4099, None), (1 << 16, 0.0)])
def test_fused_lbfgs_matches_torch(n, clamp):
    A, b = _problem(n, 256)
    key = 'projector.active_data'

    def render(vars_):
        return A @ vars_[key]

    def loss_step(vol, dvol, alpha, p):
        r = vol + alpha * dvol - b
        return (r * r).sum()

    x0 = torch.rand(n, device='cuda') * 0.1
    opts = {'torch': LinearLBFGS(render_fn=render, loss_step=loss_step),
            'fused': FusedLinearLBFGS(render_fn=render, loss_step=loss_step, clamp_min=clamp)}
    xs, hist = {}, {}
    for name, opt in opts.items():
        opt[key] = x0
        losses = []
        for _ in range(12):
            x = opt[key]
            vol = A @ x.detach()
            r = vol - b
            loss = (r * r).sum()
            x.grad = 2.0 * (A.t() @ r)
            losses.append(float(loss))
            opt.step(vol, loss)
            if clamp is not None and name == 'torch':
                opt[key] = torch.clamp_min(opt[key].detach(), clamp)
        xs[name] = opt[key].detach().cpu().numpy()
        hist[name] = losses
    np.testing.assert_allclose(hist['fused'], hist['torch'], rtol=2e-4, atol=1e-7 * hist['torch'][0])
    rel = np.linalg.norm(xs['fused'] - xs['torch']) / np.linalg.norm(xs['torch'])
    assert rel < 2e-3, rel
    assert hist['fused'][-1] < 0.5 * hist['fused'][0]


def test_loss_probes_match_single_alpha():
    """tvam_loss_threshold_probes: every step size's value equals tvam_loss_threshold's (same
    per-element arithmetic), on float4-aligned arrays and on views off the 16-byte grid."""
    from drtvam_amd.engine import loss_threshold, loss_threshold_probes
    g = torch.Generator().manual_seed(3)
    n = 1_000_003
    dose = (torch.rand(n + 1, generator=g) * 1.2).cuda()
    ddose = (torch.randn(n + 1, generator=g) * 0.3).cuda()
    target = (torch.rand(n + 1, generator=g) > 0.6).float().cuda()
    alphas = [1.0, 0.5, 0.25, 0.125, 2.0 ** -7, 3.0, 0.0, -0.5]
    args = (2, 0.85, 0.95, 1.0, 1.0, 0.5, 1.0 / n)
    for off in (0, 1):  # aligned, then every pointer 4 bytes off
        d, dd, t = dose[off:off + n], ddose[off:off + n], target[off:off + n]
        got = loss_threshold_probes(d, dd, alphas, t, *args).cpu().numpy()
        ref = np.array([float(loss_threshold(d, t, *args, ddose=dd, alpha=a)) for a in alphas])
        np.testing.assert_allclose(got, ref, rtol=1e-11)
        got3 = loss_threshold_probes(d, dd, alphas[:3], t, *args).cpu().numpy()
        np.testing.assert_allclose(got3, ref[:3], rtol=1e-11)
    with pytest.raises(Exception):
        loss_threshold_probes(dose[:n], ddose[:n], [1.0] * 9, target[:n], *args)


def test_batched_probes_same_search():
    """FusedLinearLBFGS with loss_steps (probes batched 4 per pass) takes the same step sizes,
    probe counts and losses as the one-probe-at-a-time line search (lbfgs.py:255-268), including
    searches longer than one batch."""
    A, b = _problem(4096, 256, seed=5)
    A = A * 30.0  # the first steps overshoot by far: long backtracking
    key = 'projector.active_data'

    def render(vars_):
        return A @ vars_[key]

    def loss_step(vol, dvol, alpha, p):
        r = vol + alpha * dvol - b
        return (r * r).sum().to(torch.float64)

    def loss_steps(vol, dvol, alphas, p):
        return torch.stack([loss_step(vol, dvol, a, p) for a in alphas])

    x0 = torch.rand(4096, device='cuda') * 0.1
    runs = {}
    for name, ls in (('one', None), ('batched', loss_steps)):
        opt = FusedLinearLBFGS(render_fn=render, loss_step=loss_step, clamp_min=0.0, loss_steps=ls)
        opt[key] = x0
        trace = []
        for _ in range(10):
            x = opt[key]
            vol = A @ x.detach()
            r = vol - b
            x.grad = 2.0 * (A.t() @ r)
            opt.step(vol, (r * r).sum())
            trace.append((opt.last_alpha, opt.last_search_steps, float(((A @ opt[key].detach() - b) ** 2).sum())))
        runs[name] = trace
    assert [t[:2] for t in runs['batched']] == [t[:2] for t in runs['one']]
    np.testing.assert_allclose([t[2] for t in runs['batched']], [t[2] for t in runs['one']], rtol=1e-6)
    assert max(t[1] for t in runs['one']) > FusedLinearLBFGS.probe_batch  # a search spanning batches


@pytest.mark.parametrize("is_new", [False, True])
def test_device_recursion_matches_host(is_new):
    """tvam_lbfgs_coef (the two-loop recursion on one device lane) against its host restatement
    (tests/test_lbfgs_fused.py NumpyVecLib.tvam_lbfgs_coef) on the dots of a real history pass over
    ring slots out of order; the coefficients bit-identical, then tvam_lbfgs_direction_dev against
    tvam_lbfgs_direction with those coefficients by value (bit-identical directions)."""
    import ctypes
    from drtvam_amd import _abi
    from test_lbfgs_fused import NumpyVecLib
    lib = _abi.load_library()
    n, m = 1 << 15, 7
    gen = torch.Generator().manual_seed(11)
    P = torch.randn(2, n, generator=gen).cuda()
    G = torch.randn(2, n, generator=gen).cuda()
    S = torch.randn(m, n, generator=gen).cuda() * 0.1
    Y = S * 0.5 + torch.randn(m, n, generator=gen).cuda() * 0.05  # s.y > 0
    slots = [3, 0, 5, 1]  # retained pairs, oldest first
    new_slot = 6
    h = len(slots)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())
    Sp = (ctypes.c_void_p * m)(*[S[j].data_ptr() for j in slots])
    Yp = (ctypes.c_void_p * m)(*[Y[j].data_ptr() for j in slots])
    work = torch.empty(_abi.LBFGS_WORK_DOUBLES, dtype=torch.float64, device='cuda')
    dots = torch.empty(5 * (m + 1) + 1, dtype=torch.float64, device='cuda')
    gram = torch.zeros(128, dtype=torch.float64)
    for a in range(m):  # the retained pairs' entries, as earlier steps stored them
        for b in range(m):
            gram[a * 8 + b] = float(torch.dot(S[a].double(), Y[b].double()))
            gram[64 + a * 8 + b] = float(torch.dot(Y[a].double(), Y[b].double()))
    stream = torch.cuda.current_stream().cuda_stream
    _abi.check(lib.tvam_lbfgs_history(n, ptr(P[1]) if is_new else None, ptr(P[0]) if is_new else None, ptr(G[1]),
                                      ptr(G[0]) if is_new else None, h, Sp, Yp,
                                      ptr(S[new_slot]) if is_new else None, ptr(Y[new_slot]) if is_new else None,
                                      ptr(work), ptr(dots), stream))
    order = slots + ([new_slot] if is_new else [])
    H = len(order)
    order_c = (ctypes.c_int32 * 8)(*order)
    gram_d = gram.cuda()
    coef = torch.zeros(17, dtype=torch.float32, device='cuda')
    gdz = torch.zeros(1, dtype=torch.float64, device='cuda')
    _abi.check(lib.tvam_lbfgs_coef(H, int(is_new), 0, order_c, ptr(dots), ptr(gram_d), ptr(coef), ptr(gdz), stream))
    # host restatement on the same dots and Gram entries
    dots_h, gram_h = dots.cpu(), gram.clone()
    coef_h = torch.zeros(17, dtype=torch.float32)
    gdz_h = torch.zeros(1, dtype=torch.float64)
    NumpyVecLib().tvam_lbfgs_coef(H, int(is_new), 0, order_c, dots_h.data_ptr(), gram_h.data_ptr(),
                                  coef_h.data_ptr(), gdz_h.data_ptr(), None)
    assert torch.equal(coef.cpu(), coef_h)
    assert torch.equal(gram_d.cpu(), gram_h)
    np.testing.assert_allclose(gdz.item(), gdz_h.item(), rtol=1e-12)
    # the direction from device coefficients == the direction from the same values by value
    S2 = (ctypes.c_void_p * 8)(*[S[j].data_ptr() for j in order])
    Y2 = (ctypes.c_void_p * 8)(*[Y[j].data_ptr() for j in order])
    d_dev = torch.empty(n, device='cuda')
    d_val = torch.empty(n, device='cuda')
    _abi.check(lib.tvam_lbfgs_direction_dev(n, ptr(G[1]), H, S2, Y2, ptr(coef), ptr(d_dev), stream))
    c = coef_h.numpy()
    cs = (ctypes.c_float * 8)(*[float(v) for v in c[1:1 + H]])
    cy = (ctypes.c_float * 8)(*[float(v) for v in c[9:9 + H]])
    _abi.check(lib.tvam_lbfgs_direction(n, ptr(G[1]), H, S2, Y2, float(c[0]), cs, cy, ptr(d_val), stream))
    assert torch.equal(d_dev, d_val)
    # and g.d of the direction itself
    np.testing.assert_allclose(gdz.item(), float(torch.dot(G[1].double(), d_dev.double())), rtol=1e-4)


def test_armijo_kernel_matches_host_decision():
    """tvam_lbfgs_armijo (the first probe batch decided on one device lane) against the host loop of
    FusedLinearLBFGS.step (lbfgs.py:256-266): the same step size, bit for bit, on probes placed at
    and around the Armijo bound (ties included), with a device loss (divided over ranks) and a host
    loss; 0 when no probe passes."""
    import ctypes
    from drtvam_amd import _abi
    lib = _abi.load_library()
    stream = torch.cuda.current_stream().cuda_stream
    c1 = 1e-4
    rng = np.random.default_rng(7)
    alpha = torch.empty(1, dtype=torch.float32, device='cuda')
    for case in range(200):
        nb = int(rng.integers(1, 5))
        loss = float(rng.uniform(0.1, 10.0)) * (1.0 if case % 5 else 0.0)
        gdz = -float(rng.uniform(0.0, 5.0))
        div = float(rng.choice([1.0, 2.0, 8.0]))
        lv = (loss * div) / div
        bound = [lv + c1 * (0.5 ** j) * gdz for j in range(nb)]
        kind = rng.integers(0, 3, size=nb)  # above / at / below the bound
        probes = [b + (1.0 if k == 0 else (0.0 if k == 1 else -1e-3)) * (abs(b) + 1.0) for b, k in zip(bound, kind)]
        host = 0.0
        for j, f in enumerate(probes):
            if f <= lv + c1 * (1.0 * 0.5 ** j) * (0.0 + gdz):
                host = 0.5 ** j
                break
        pr = torch.tensor(probes, dtype=torch.float64, device='cuda')
        gd = torch.tensor([gdz], dtype=torch.float64, device='cuda')
        if case % 2:
            ld = torch.tensor([loss * div], dtype=torch.float64, device='cuda')
            _abi.check(lib.tvam_lbfgs_armijo(nb, 1.0, pr.data_ptr(), ld.data_ptr(), 0.0, div, gd.data_ptr(), c1,
                                             alpha.data_ptr(), None, stream))
        else:
            _abi.check(lib.tvam_lbfgs_armijo(nb, 1.0, pr.data_ptr(), None, lv, 1.0, gd.data_ptr(), c1,
                                             alpha.data_ptr(), None, stream))
        assert float(alpha.item()) == host, (case, probes, bound)
    with pytest.raises(ValueError):
        _abi.check(lib.tvam_lbfgs_armijo(0, 1.0, pr.data_ptr(), None, 1.0, 1.0, gd.data_ptr(), c1,
                                         alpha.data_ptr(), None, stream))


@pytest.mark.parametrize("scale", [1.0, 30.0])
def test_speculative_update_is_the_host_update(scale):
    """FusedLinearLBFGS.step with the update launched behind the first probes (tvam_lbfgs_armijo +
    tvam_axpy_clamp_dev, the host reading the probes on a side stream) against the host-decided
    update: identical step sizes, probe counts and patterns, bit for bit; scale 30 overshoots, so
    searches outlast the first batch and the speculative update is discarded."""
    A, b = _problem(8192, 256, seed=9)
    A = A * scale
    key = 'projector.active_data'

    def render(vars_):
        return A @ vars_[key]

    def loss_steps(vol, dvol, alphas, p):
        return torch.stack([((vol + a * dvol - b) ** 2).sum().to(torch.float64) for a in alphas])

    x0 = torch.rand(8192, device='cuda') * 0.1
    runs = {}
    for spec in (False, True):
        opt = FusedLinearLBFGS(render_fn=render, clamp_min=0.0, loss_steps=loss_steps)
        opt.speculate = spec
        opt[key] = x0
        trace, xs = [], []
        for _ in range(10):
            x = opt[key]
            vol = A @ x.detach()
            r = vol - b
            x.grad = 2.0 * (A.t() @ r)
            opt.step(vol, None, loss_dev=(r * r).sum().to(torch.float64))
            trace.append((opt.last_alpha, opt.last_search_steps))
            xs.append(opt[key].detach().clone())
        runs[spec] = (trace, xs)
    assert runs[True][0] == runs[False][0]
    for a, c in zip(runs[True][1], runs[False][1]):
        assert torch.equal(a, c)
    if scale > 1.0:
        assert max(t[1] for t in runs[True][0]) > FusedLinearLBFGS.probe_batch


def test_target_mask_loss_is_the_f32_target_loss():
    """tvam_loss_threshold(_probes)_mask (the object test read from the target's bit mask) against the
    f32-target kernels: values to 1e-12 (the blocks' f64 partials meet in atomics, in any order)
    and the same gradient bit for bit, on the whole film and on slabs at
    bit offsets that are and are not multiples of 4 and 32 (scalar and float4 paths); greyscale
    targets (> 0 = object); and ThresholdedLoss rebuilds its cached mask when the target is written."""
    from drtvam_amd.engine import loss_threshold, loss_threshold_probes, target_mask
    from drtvam_amd.loss import ThresholdedLoss
    g = torch.Generator().manual_seed(4)
    n = 64 * 1000 + 13
    dose = (torch.rand(n, generator=g) * 1.3).cuda()
    ddose = (torch.randn(n, generator=g) * 0.2).cuda()
    tgt = torch.rand(n, generator=g)
    tgt = torch.where(tgt > 0.55, tgt, torch.where(tgt > 0.5, -tgt, torch.zeros_like(tgt))).cuda()
    mask = target_mask(tgt)
    bits = torch.tensor([(int(w) & 0xffffffff) >> j & 1 for w in mask.cpu().tolist() for j in range(32)][:n])
    assert torch.equal(bits.bool(), (tgt > 0).cpu())
    args = (2, 0.85, 0.95, 1.0, 1.3, 0.7, 1.0 / n)
    alphas = [1.0, 0.5, 0.25, 0.125]
    for z0, z1 in ((0, n), (32 * 500, 32 * 1500), (4 * 301, n - 7), (5, 64 * 999)):
        d, dd, t = dose[z0:z1], ddose[z0:z1], tgt[z0:z1]
        g0, g1 = torch.empty_like(d), torch.empty_like(d)
        v0 = loss_threshold(d, t, *args, grad=g0)
        v1 = loss_threshold(d, t, *args, grad=g1, mask=mask, mask_bit0=z0)
        assert float(v0) == pytest.approx(float(v1), rel=1e-12)
        assert torch.equal(g0, g1)
        p0 = loss_threshold_probes(d, dd, alphas, t, *args)
        p1 = loss_threshold_probes(d, dd, alphas, t, *args, mask=mask, mask_bit0=z0)
        torch.testing.assert_close(p0, p1, rtol=1e-12, atol=0)
        s0 = loss_threshold(d, t, *args, ddose=dd, alpha=0.3)
        s1 = loss_threshold(d, t, *args, ddose=dd, alpha=0.3, mask=mask, mask_bit0=z0)
        assert float(s0) == pytest.approx(float(s1), rel=1e-12)
    with pytest.raises(ValueError):
        loss_threshold(dose, tgt, *args, mask=mask, mask_bit0=32)
    lf = ThresholdedLoss({"K": 2, "tl": 0.85, "tu": 0.95})
    grad = torch.empty_like(dose)
    a = float(lf.fused_value_grad(dose, tgt, None, grad))
    tgt[: n // 2] = 1.0  # in place: the cached mask is rebuilt
    b = float(lf.fused_value_grad(dose, tgt, None, grad))
    ref = float(loss_threshold(dose, tgt, 2, lf.tl, lf.tu, 1.0, 1.0, 1.0, 1.0))  # sum reduction
    assert b == pytest.approx(ref, rel=1e-12) and abs(a - b) > 1e-6 * abs(b)


def test_history_with_precomputed_s():
    """tvam_lbfgs_history with the new pair's s already in its slot (p_old NULL, g_old given: written by
    tvam_axpy_clamp_dev's s_out) against the pass that forms s = p - p_old: the same dots and y, bit for
    bit, and the update's s_out equal to out - p."""
    import ctypes
    from drtvam_amd import _abi
    lib = _abi.load_library()
    n, m = (1 << 16) + 12, 7
    gen = torch.Generator().manual_seed(21)
    P0 = torch.rand(n, generator=gen).cuda()
    D = torch.randn(n, generator=gen).cuda()
    G = torch.randn(2, n, generator=gen).cuda()
    S = torch.randn(m, n, generator=gen).cuda() * 0.1
    Y = S * 0.5 + torch.randn(m, n, generator=gen).cuda() * 0.05
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())
    stream = torch.cuda.current_stream().cuda_stream
    alpha = torch.tensor([0.25], dtype=torch.float32, device='cuda')
    P1 = torch.empty_like(P0)
    s_pre = torch.empty_like(P0)
    _abi.check(lib.tvam_axpy_clamp_dev(n, ptr(P0), ptr(alpha), ptr(D), 0.0, ptr(P1), ptr(s_pre), stream))
    assert torch.equal(s_pre, P1 - P0)
    assert torch.equal(P1, torch.clamp_min(P0 + 0.25 * D, 0.0))
    h = 4
    Sp = (ctypes.c_void_p * m)(*[S[j].data_ptr() for j in range(h)])
    Yp = (ctypes.c_void_p * m)(*[Y[j].data_ptr() for j in range(h)])
    work = torch.empty(_abi.LBFGS_WORK_DOUBLES, dtype=torch.float64, device='cuda')
    res = []
    for pre in (False, True):
        s_new = s_pre.clone() if pre else torch.empty_like(P0)
        y_new = torch.empty_like(P0)
        dots = torch.zeros(5 * (m + 1) + 1, dtype=torch.float64, device='cuda')
        _abi.check(lib.tvam_lbfgs_history(n, None if pre else ptr(P1), None if pre else ptr(P0), ptr(G[1]), ptr(G[0]),
                                          h, Sp, Yp, ptr(s_new), ptr(y_new), ptr(work), ptr(dots), stream))
        res.append((s_new, y_new, dots))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    assert torch.equal(res[0][2], res[1][2])
    with pytest.raises(ValueError):  # g_old without p_old in the row-band variant
        _abi.check(lib.tvam_lbfgs_history_rows(1, 64, 64, 0, None, None, ptr(G[1]), ptr(G[0]), h, Sp, Yp,
                                               ptr(s_pre), ptr(P1), ptr(work), ptr(res[0][2]), stream))
