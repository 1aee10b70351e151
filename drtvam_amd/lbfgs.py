"""Linear L-BFGS (mirror of drtvam/lbfgs.py:146-275) on torch tensors.

The forward model is linear in the patterns, so the line search never
re-renders: it renders the search direction once (``render_fn``, lbfgs.py:248)
and probes ``loss_fn(vol + alpha*dvol)`` with backtracking Armijo
(lbfgs.py:256-266).  History vectors, dots and axpys stay on the device; the
only host syncs are the Armijo decisions (as in the reference, lbfgs.py:263).

``dot`` may be replaced (e.g. by an all-reduced dot over angle shards) and
``loss_step`` may evaluate ``loss(vol + alpha*dvol)`` without materialising it.
"""
from __future__ import annotations

import torch


def _dot(a, b):
    return torch.dot(a, b)


class LinearLBFGS:
    def __init__(self, lr=1.0, m=5, params=None, render_fn=None, loss_fn=None, search_it=20, dot=None,
                 loss_step=None):
        self.lr = lr
        self.m = m
        self.p_old = {}
        self.g_old = {}
        self.s = {}
        self.y = {}
        self.ys = {}
        self.t = {}
        self.render_fn = render_fn
        self.loss_fn = loss_fn
        self.loss_step = loss_step
        self.search_it = search_it
        self.dot = dot or _dot
        self.variables = {}
        self.last_alpha = None
        self.last_search_steps = 0
        if params:
            for k, v in params.items():
                self[k] = v

    # mi.ad.Optimizer-style access
    def __setitem__(self, key, value):
        v = value.detach().clone() if isinstance(value, torch.Tensor) else torch.as_tensor(value)
        v.requires_grad_(True)
        self.variables[key] = v

    def __getitem__(self, key):
        return self.variables[key]

    def keys(self):
        return self.variables.keys()

    def items(self):
        return self.variables.items()

    def reset(self, k):
        self.s[k] = []
        self.y[k] = []
        self.ys[k] = []
        self.t[k] = 0

    def update_history(self, k):
        if self.t[k] > self.m:
            self.s[k].pop(0)
            self.y[k].pop(0)
            self.ys[k].pop(0)
        p = self.variables[k].detach().reshape(-1)
        g_p = self.variables[k].grad.detach().reshape(-1)
        if self.t[k] > 0:
            self.s[k].append(p - self.p_old[k])
            self.y[k].append(g_p - self.g_old[k])
            self.ys[k].append(self.dot(self.y[k][-1], self.s[k][-1]))
        self.p_old[k] = p.clone()
        self.g_old[k] = g_p.clone()
        self.t[k] += 1

    @torch.no_grad()
    def step(self, vol, loss):
        search_dirs = {}
        for k, p in self.variables.items():
            if k not in self.s:
                self.reset(k)
            self.update_history(k)
            q = p.grad.detach().reshape(-1).clone()
            s, y, ys = self.s[k], self.y[k], self.ys[k]
            hist_size = len(s)
            alphas = [None] * hist_size
            for i in range(hist_size - 1, -1, -1):
                rho = 1.0 / ys[i]
                a = rho * self.dot(s[i], q)
                q.sub_(a * y[i])
                alphas[i] = a
            gamma = 1.0 if self.t[k] == 1 else ys[-1] / self.dot(y[-1], y[-1])
            z = gamma * q
            for i in range(hist_size):
                rho = 1.0 / ys[i]
                b = rho * self.dot(y[i], z)
                z.add_((alphas[i] - b) * s[i])
            search_dirs[k] = -z

        c1 = 1e-4
        params = {k: search_dirs[k].reshape(self.variables[k].shape) for k in self.variables}
        dvol = self.render_fn(params)

        g_dot_z = None
        for k in params:
            v = self.dot(self.g_old[k], search_dirs[k])
            g_dot_z = v if g_dot_z is None else g_dot_z + v
        g_dot_z = float(g_dot_z)
        loss_v = float(loss)
        key = 'projector.active_data' if 'projector.active_data' in params else next(iter(params))
        alpha = 1.0
        steps = 0
        for _ in range(self.search_it):
            steps += 1
            if self.loss_step is not None:
                f_new = self.loss_step(vol, dvol, alpha, params[key])
            else:
                f_new = self.loss_fn(vol + alpha * dvol, params[key])
            if float(f_new) <= loss_v + c1 * alpha * g_dot_z:
                break
            alpha *= 0.5
        self.last_alpha = alpha
        self.last_search_steps = steps

        for k, p in self.variables.items():
            newp = (p.detach() + alpha * search_dirs[k].reshape(p.shape))
            self.variables[k] = newp.requires_grad_(True)
