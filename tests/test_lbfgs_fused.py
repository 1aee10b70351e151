"""FusedLinearLBFGS bookkeeping (ring slots, eviction, Gram updates, scalar
two-loop recursion) against the torch LinearLBFGS restatement of
lbfgs.py:146-275, on CPU: the three libtvam vector kernels are replaced by a
numpy stand-in reading the same pointers (the GPU kernels themselves are
checked in tests/test_gpu_lbfgs.py)."""
import ctypes

import numpy as np
import torch

from drtvam_amd import _abi
from drtvam_amd.lbfgs import FusedLinearLBFGS, LinearLBFGS


def _view(ptr, n, ctype=ctypes.c_float):
    return np.ctypeslib.as_array((ctype * n).from_address(int(ptr)))


class NumpyVecLib:
    """Host restatement of tvam_lbfgs_history / _coef / _direction(_dev) / tvam_axpy_clamp (include/tvam.h)."""

    def tvam_lbfgs_history(self, n, p, p_old, g, g_old, h, S, Y, s_new, y_new, work, dots, stream):
        gv = _view(g, n).astype(np.float64)
        Sv = [_view(S[j], n).astype(np.float64) for j in range(h)]
        Yv = [_view(Y[j], n).astype(np.float64) for j in range(h)]
        out = []
        if p_old is not None:
            sn = (_view(p, n) - _view(p_old, n)).astype(np.float32)
            yn = (_view(g, n) - _view(g_old, n)).astype(np.float32)
            _view(s_new, n)[:] = sn
            _view(y_new, n)[:] = yn
            Sv.append(sn.astype(np.float64))
            Yv.append(yn.astype(np.float64))
            out += [s @ gv for s in Sv] + [y @ gv for y in Yv]
            out += [Sv[-1] @ y for y in Yv] + [s @ Yv[-1] for s in Sv] + [Yv[-1] @ y for y in Yv]
        else:
            out += [s @ gv for s in Sv] + [y @ gv for y in Yv]
        out.append(gv @ gv)
        _view(dots, len(out), ctypes.c_double)[:] = out
        return 0

    def tvam_lbfgs_direction(self, n, g, h, S, Y, cg, cs, cy, d, stream):
        r = cg * _view(g, n).astype(np.float64)
        for j in range(h):
            r += cs[j] * _view(S[j], n) + cy[j] * _view(Y[j], n)
        _view(d, n)[:] = r.astype(np.float32)
        return 0

    def tvam_lbfgs_coef(self, h, is_new, first, order, dots, gram, coef, gdz, stream):
        """The device recursion (tvam_vec.hip tvam_lbfgs_coef_kernel): Gram entries by ring slot."""
        o = [order[j] for j in range(h)]
        nd = 5 * h + 1 if is_new else 2 * h + 1
        dv = _view(dots, nd, ctypes.c_double).copy()
        gr = _view(gram, 128, ctypes.c_double)
        SY, YY = gr[:64].reshape(8, 8), gr[64:].reshape(8, 8)
        Sg, Yg, gg = dv[:h], dv[h:2 * h], dv[nd - 1]
        if is_new:
            sl = o[-1]
            for j, sj in enumerate(o):
                SY[sl, sj] = dv[2 * h + j]
                SY[sj, sl] = dv[3 * h + j]
                YY[sl, sj] = YY[sj, sl] = dv[4 * h + j]
        a = np.zeros(h)
        for i in range(h - 1, -1, -1):
            a[i] = (Sg[i] - sum(a[j] * SY[o[i], o[j]] for j in range(i + 1, h))) / SY[o[i], o[i]]
        gamma = 1.0 if (first or h == 0) else SY[o[-1], o[-1]] / YY[o[-1], o[-1]]
        b = np.zeros(h)
        for i in range(h):
            yz = gamma * (Yg[i] - sum(a[j] * YY[o[i], o[j]] for j in range(h)))
            yz += sum((a[j] - b[j]) * SY[o[j], o[i]] for j in range(i))
            b[i] = yz / SY[o[i], o[i]]
        cs, cy = -(a - b), gamma * a
        c = _view(coef, 17)
        c[0] = -gamma
        c[1:1 + h] = cs
        c[9:9 + h] = cy
        _view(gdz, 1, ctypes.c_double)[0] = -gamma * gg + float(np.dot(cs, Sg)) + float(np.dot(cy, Yg))
        return 0

    def tvam_lbfgs_direction_dev(self, n, g, h, S, Y, coef, d, stream):
        c = _view(coef, 17)
        return self.tvam_lbfgs_direction(n, g, h, S, Y, float(c[0]), c[1:1 + h], c[9:9 + h], d, stream)

    def tvam_axpy_clamp(self, n, p, alpha, d, lo, out, stream):
        _view(out, n)[:] = np.maximum(_view(p, n) + np.float32(alpha) * _view(d, n), np.float32(lo))
        return 0


def test_fused_bookkeeping_matches_torch(monkeypatch):
    monkeypatch.setattr(FusedLinearLBFGS, "_lib", lambda self: NumpyVecLib())
    monkeypatch.setattr(_abi, "check", lambda rc: rc)
    n, k = 2000, 300
    g = torch.Generator().manual_seed(0)
    A = torch.randn(k, n, generator=g) / n ** 0.5
    b = torch.randn(k, generator=g)
    key = 'projector.active_data'

    def render(vars_):
        return A @ vars_[key]

    def loss_step(vol, dvol, alpha, p):
        r = vol + alpha * dvol - b
        return (r * r).sum()

    x0 = torch.rand(n, generator=g) * 0.1
    res = {}
    for name, cls in (("torch", LinearLBFGS), ("fused", FusedLinearLBFGS)):
        opt = cls(render_fn=render, loss_step=loss_step)
        opt[key] = x0
        losses, alphas = [], []
        for _ in range(12):  # > m + 1 steps: the ring evicts
            x = opt[key]
            vol = A @ x.detach()
            r = vol - b
            loss = (r * r).sum()
            x.grad = 2.0 * (A.t() @ r)
            losses.append(float(loss))
            opt.step(vol, loss)
            alphas.append(opt.last_alpha)
        res[name] = (np.array(losses), alphas, opt[key].detach().numpy())
    # fp64 Gram dots vs the reference's fp32 dots: agreement to ~1e-7 of the initial loss
    np.testing.assert_allclose(res["fused"][0], res["torch"][0], rtol=1e-4, atol=1e-7 * res["torch"][0][0])
    assert res["fused"][1] == res["torch"][1]
    np.testing.assert_allclose(res["fused"][2], res["torch"][2], rtol=1e-3, atol=1e-5)
