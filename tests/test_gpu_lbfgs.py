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
