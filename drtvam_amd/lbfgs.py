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

import ctypes
import time

import torch


def _dot(a, b):
    return torch.dot(a, b)



def _abi_work_doubles():
    from ._abi import LBFGS_WORK_DOUBLES
    return LBFGS_WORK_DOUBLES

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


class DirectionPipeline:
    """Slab bands of one optimiser iteration for FusedLinearLBFGS.step_pipelined (one variable,
    dense patterns [nseg][rows][cols], CUDA): parts = [(row0, row1, z0, z1), ...] tile the rows and
    the film, and film slices [z0, z1) depend only on pattern rows [row0, row1) (planar rays: a
    row's rays stay in its slice).  The projections of a band run on the current stream, the
    HBM-bound vector passes of the neighbouring band on ``side``, so each hides under the other.
    Callbacks: render_part(x, z0, z1, out) (forward of slices [z0, z1) into out), probe_part(vol,
    dvol, alphas, z0, z1) (f64 device losses of that slab, no all-reduce), reduce(t) (sum over
    slab ranks, or identity), new_dose()."""

    def __init__(self, nseg, rows, cols, parts, render_part, probe_part, reduce, new_dose):
        self.nseg, self.rows, self.cols = nseg, rows, cols
        self.parts = parts
        self.render_part = render_part
        self.probe_part = probe_part
        self.reduce = reduce
        self.new_dose = new_dose
        self._side = None

    def side(self, dev):
        if self._side is None:
            self._side = torch.cuda.Stream(dev)
        return self._side


def _aligned(v):
    """v itself when 16-byte aligned and contiguous (the fused kernels read float4), else an aligned copy."""
    return v if v.is_contiguous() and v.data_ptr() % 16 == 0 else v.clone(memory_format=torch.contiguous_format)


class FusedLinearLBFGS(LinearLBFGS):
    """LinearLBFGS with the vector work fused into three HIP passes (libtvam).

    Same algorithm as LinearLBFGS (lbfgs.py:198-275): history update, two-loop
    recursion with m pairs and gamma = s.y / y.y, one render of the search
    direction, backtracking Armijo on loss(vol + alpha dvol).  The recursion is
    evaluated on fp64 scalars from the dot products of one fused pass
    (tvam_lbfgs_history) by one device lane (tvam_lbfgs_coef, the Gram entries
    kept on the device by ring slot), the direction is one linear combination
    of g, s_i, y_i (tvam_lbfgs_direction_dev, coefficients read from the
    device), and the update p + alpha d is fused with the clamp of
    optimize.py:316-318 when ``clamp_min`` is set (tvam_axpy_clamp).  History
    pairs live in a preallocated ring of m slots.  ``allreduce`` sums the dot
    vector over angle shards (one collective per step).
    """

    probe_batch = 4  # Armijo step sizes per loss_steps pass

    def __init__(self, lr=1.0, m=5, params=None, render_fn=None, loss_fn=None, search_it=20, loss_step=None,
                 allreduce=None, clamp_min=None, loss_steps=None, pipeline=None):
        if m > 7:
            raise ValueError("FusedLinearLBFGS keeps at most 7 history pairs")
        self.allreduce = allreduce
        self.clamp_min = clamp_min
        self.loss_steps = loss_steps  # (vol, dvol, alphas, patterns) -> losses: the probes batched
        # DirectionPipeline (one variable, CUDA): the direction formed in row bands, each band's
        # forward (its film slices) rendered on a second stream while the next band is formed
        self.pipeline = pipeline
        self.state = {}
        super().__init__(lr=lr, m=m, params=params, render_fn=render_fn, loss_fn=loss_fn, search_it=search_it,
                         loss_step=loss_step)

    def __setitem__(self, key, value):
        v = torch.as_tensor(value).detach()
        if v.dtype != torch.float32 or not v.is_contiguous():
            v = v.to(torch.float32).contiguous()
        v.requires_grad_(True)
        self.variables[key] = v

    def reset(self, k):
        self.state.pop(k, None)

    def _lib(self):
        from . import _abi
        return _abi.load_library()

    @torch.no_grad()
    def step_pipelined(self, vol, loss_parts, loss_summed, grad_ready):
        """step() for one variable under self.pipeline, the gradient arriving in row bands: grad_ready
        = [(event, row0, row1), ...], band k of p.grad final once event k (recorded on the current
        stream) has fired; loss_parts = the slab bands' loss values (f64 device scalars, on the side
        stream).  The same algorithm and kernels as step(), banded: the history pass of band k
        (tvam_lbfgs_history_rows, its dots summed over the bands in band order) runs on the side
        stream while band k + 1's adjoint runs; after the recursion, direction band k
        (tvam_lbfgs_direction_rows) precedes band k's render on the current stream, and band k's
        first four Armijo probes follow it on the side stream.  One host read (loss, g.d, probes)."""
        from . import _abi
        lib = self._lib()
        pipe = self.pipeline
        (k, p), = self.variables.items()
        dev0 = p.device
        side = pipe.side(dev0)
        K = len(pipe.parts)
        # state created here is zero-filled on the side stream, which writes it next (the fills
        # must not race the side stream's history / coefficient kernels)
        with torch.cuda.stream(side):
            st = self._st(k, p)
            if st.get('dots_b') is None or st['dots_b'].shape[0] != K:
                st['dots_b'] = torch.zeros((K, 64), dtype=torch.float64, device=dev0)
        pf = _aligned(p.detach().reshape(-1))
        g = p.grad.detach().reshape(-1)
        if not (g.is_contiguous() and g.data_ptr() % 16 == 0):
            raise ValueError("step_pipelined: the gradient must be a 16-byte aligned contiguous tensor")
        dev = pf.device
        main = torch.cuda.current_stream(dev)
        ss = side.cuda_stream
        R, C = pipe.rows, pipe.cols
        new = st['t'] > 0
        if new and len(st['slots']) == self.m:  # evict the oldest pair (lbfgs.py:214-217)
            st['free'].append(st['slots'].pop(0))
        kept = list(st['slots'])
        h = len(kept)
        S_ptrs = (ctypes.c_void_p * max(h, 1))(*[st['S_ptr'][j] for j in kept])
        Y_ptrs = (ctypes.c_void_p * max(h, 1))(*[st['Y_ptr'][j] for j in kept])
        slot = st['free'][0] if new else None
        nd = 5 * (h + 1) + 1 if new else 2 * h + 1
        dots_b = st['dots_b']
        with torch.cuda.stream(side):
            dots_b.zero_()
            for ev, r0, r1 in grad_ready:
                side.wait_event(ev)
                b = [i for i, q in enumerate(pipe.parts) if q[0] == r0][0]
                if r1 > r0:
                    _abi.check(lib.tvam_lbfgs_history_rows(
                        pipe.nseg, (r1 - r0) * C, R * C, r0 * C, pf.data_ptr() if new else None,
                        st['p_old'].data_ptr() if new else None, g.data_ptr(), st['g_old'].data_ptr() if new else None,
                        h, S_ptrs, Y_ptrs, st['S_ptr'][slot] if new else None, st['Y_ptr'][slot] if new else None,
                        st['work'].data_ptr(), dots_b[b].data_ptr(), ss))
            dots = dots_b[:, :nd].sum(0)
            with_loss = loss_parts is not None
            if with_loss:
                lsum = loss_parts[0]
                for v in loss_parts[1:]:
                    lsum = lsum + v
                dots = torch.cat([dots, lsum.reshape(1).to(torch.float64)])
            if self.allreduce is not None:
                dots = self.allreduce(dots.clone())
            loss_cell = dots[nd:nd + 1] if with_loss else None
            if new:
                st['free'].pop(0)
                st['slots'].append(slot)
            order = st['slots']
            H = len(order)
            st['p_old'], st['g_old'] = pf, g
            st['t'] += 1
            gdz = torch.empty(1, dtype=torch.float64, device=dev)
            order_c = (ctypes.c_int32 * max(H, 1))(*order)
            _abi.check(lib.tvam_lbfgs_coef(H, int(new), int(st['t'] == 1), order_c, dots.data_ptr(),
                                           st['gram'].data_ptr(), st['coef'].data_ptr(), gdz.data_ptr(), ss))
            d = torch.empty_like(g)
            d.record_stream(main)  # rendered and stepped along on the current stream
            S2 = (ctypes.c_void_p * max(H, 1))(*[st['S_ptr'][j] for j in order])
            Y2 = (ctypes.c_void_p * max(H, 1))(*[st['Y_ptr'][j] for j in order])
        dvol = pipe.new_dose()
        alphas = [0.5 ** j for j in range(min(self.probe_batch, self.search_it))]
        probes = []
        for r0, r1, z0, z1 in pipe.parts:
            with torch.cuda.stream(side):
                if r1 > r0:
                    _abi.check(lib.tvam_lbfgs_direction_rows(pipe.nseg, (r1 - r0) * C, R * C, r0 * C, g.data_ptr(), H,
                                                             S2, Y2, st['coef'].data_ptr(), d.data_ptr(), ss))
                ev = torch.cuda.Event()
                ev.record(side)
            main.wait_event(ev)
            if z1 > z0:
                pipe.render_part(d, z0, z1, dvol)
                evf = torch.cuda.Event()
                evf.record(main)
                side.wait_event(evf)
                with torch.cuda.stream(side):
                    probes.append(pipe.probe_part(vol, dvol, alphas, z0, z1))
        with torch.cuda.stream(side):
            pv = probes[0]
            for v in probes[1:]:
                pv = pv + v
            pv = pipe.reduce(pv)
            parts = ([loss_cell] if loss_cell is not None else []) + [gdz, pv]
            hv = torch.cat([t.reshape(-1).to(torch.float64) for t in parts]).cpu().tolist()
        main.wait_stream(side)
        loss_v = hv.pop(0) if loss_cell is not None else None
        if loss_cell is not None and self.allreduce is not None and not loss_summed:
            import torch.distributed as _d
            loss_v = loss_v / _d.get_world_size()
        gdz_v = hv.pop(0)
        if loss_cell is not None and loss_v == 0.0:  # converged (optimize.py:305-307): no update
            return loss_v
        # the backtracking sequence of step(): the first batch came with the read
        c1 = 1e-4
        params = {k: d.reshape(p.shape)}
        alpha, steps, done, fv = 1.0, 0, False, hv
        while True:
            for a, f_new in zip(alphas, fv):
                steps += 1
                alpha = a
                if f_new <= loss_v + c1 * a * gdz_v:
                    done = True
                    break
            if done:
                break
            alpha *= 0.5
            if steps >= self.search_it:
                break
            nb = min(self.probe_batch, self.search_it - steps)
            alphas = [alpha * 0.5 ** j for j in range(nb)]
            fv = self.loss_steps(vol, dvol, alphas, params[k]).cpu().tolist()
        self.last_alpha = alpha
        self.last_search_steps = steps
        lo = -float('inf') if self.clamp_min is None else float(self.clamp_min)
        out = torch.empty_like(pf)
        _abi.check(lib.tvam_axpy_clamp(pf.numel(), pf.data_ptr(), float(alpha), d.data_ptr(), lo, out.data_ptr(),
                                       self._stream(dev)))
        self.variables[k] = out.reshape(p.shape).requires_grad_(True)
        return loss_v

    speculate = True  # decide the first probe batch on the device and launch the update behind it

    def _speculative_update(self, fd, nb, c1, loss, loss_cell, gdz, loss_summed, search, lo):
        """The first probe batch decided on the device (tvam_lbfgs_armijo) and the update p + alpha d
        with that alpha (tvam_axpy_clamp_dev) launched behind it, the host reading the decision's
        report (loss, g.d, probes, alpha) from pinned memory as soon as the decision kernel is done:
        the update runs while the host decides and launches the next iteration, where the GPU
        idled through the read before.  Returns ((update, device alpha), loss, g.d, probes) with
        the loss and g.d formed as host_scalars forms them; the caller keeps the update only when
        its own decision took the same alpha from this batch."""
        from . import _abi
        lib = self._lib()
        (k, p), = self.variables.items()
        pf = _aligned(p.detach().reshape(-1))
        dev = pf.device
        main = torch.cuda.current_stream(dev)
        div = 1.0
        divided = loss_cell is not None and self.allreduce is not None and not loss_summed
        if divided:
            import torch.distributed as _d
            div = float(_d.get_world_size())
        rep = getattr(self, '_report', None)
        if rep is None or rep.numel() < 4 + nb:
            rep = self._report = torch.zeros(4 + max(nb, self.probe_batch), dtype=torch.float64, pin_memory=True)
            self._report_np = rep.numpy()
            self._alpha_dev = torch.empty(1, dtype=torch.float32, device=dev)
        rnp = self._report_np
        rnp[3 + nb] = 0.0  # the kernel's done flag
        alpha_dev = self._alpha_dev
        if alpha_dev.device != dev:
            alpha_dev = self._alpha_dev = torch.empty(1, dtype=torch.float32, device=dev)
        loss_host = float(loss) if loss_cell is None else 0.0
        fdc = fd.contiguous()
        _abi.check(lib.tvam_lbfgs_armijo(nb, 1.0, fdc.data_ptr(), loss_cell.data_ptr() if loss_cell is not None else None,
                                         loss_host, div, gdz.data_ptr(), c1, alpha_dev.data_ptr(), rep.data_ptr(),
                                         main.cuda_stream))
        out = torch.empty_like(pf)
        # the next step's new pair goes to the first free ring slot, or evicts the oldest: its s = out - p
        # is written there now (the slot's old pair, if any, is past its last read: this step's direction)
        st = self.state[k]
        nxt = st['free'][0] if st['free'] else st['slots'][0]
        pre = None
        if st['p_old'] is not None and st['p_old'].data_ptr() == pf.data_ptr():
            pre = {'slot': nxt, 'out': out, 'out_v': out._version, 'p': st['p_old'], 'p_v': st['p_old']._version}
        _abi.check(lib.tvam_axpy_clamp_dev(pf.numel(), pf.data_ptr(), alpha_dev.data_ptr(), search[k].data_ptr(), lo,
                                           out.data_ptr(), st['S_ptr'][nxt] if pre is not None else None,
                                           main.cuda_stream))
        # poll the done flag (an event recorded between the decision and the update would idle the GPU
        # for a few microseconds at that boundary)
        polls, t_end = 0, None
        while rnp[3 + nb] == 0.0:
            polls += 1
            if polls % 4096 == 0:
                now = time.perf_counter()
                t_end = t_end or now + 600.0  # the queue ahead of the decision: a forward and the probes
                if now > t_end:
                    raise RuntimeError("tvam_lbfgs_armijo: no report after 600 s")
        v = [float(x) for x in rnp[:3 + nb]]
        lv = v[0] / div if divided else (v[0] if loss_cell is not None else loss_host)
        return (out, v[2 + nb], pre), float(lv), 0.0 + v[1], v[2:2 + nb]

    @staticmethod
    def _stream(dev):
        return torch.cuda.current_stream(dev).cuda_stream if dev.type == 'cuda' else None

    def _st(self, k, p):
        st = self.state.get(k)
        n = p.numel()
        if st is None or st['n'] != n:
            dev = p.device
            npad = (n + 3) // 4 * 4  # 16-byte aligned rows (the kernels read float4)
            st = {'n': n, 't': 0, 'slots': [], 'free': list(range(self.m)), 'p_old': None, 'g_old': None,
                  'S': torch.empty((self.m, npad), dtype=torch.float32, device=dev)[:, :n],
                  'Y': torch.empty((self.m, npad), dtype=torch.float32, device=dev)[:, :n],
                  'work': torch.empty(_abi_work_doubles(), dtype=torch.float64, device=dev),
                  'dots': torch.empty(5 * (self.m + 1) + 1, dtype=torch.float64, device=dev),
                  # Gram entries by ring slot (s_a.y_b, then y_a.y_b; tvam_lbfgs_coef) and the direction's
                  # coefficients (cg | cs[8] | cy[8])
                  'gram': torch.zeros(2 * 64, dtype=torch.float64, device=dev),
                  'coef': torch.zeros(17, dtype=torch.float32, device=dev)}
            # device addresses of the ring's rows (plain integers: a tensor view per row and call
            # cost microseconds of host time between the dot read and the direction launch)
            st['S_ptr'] = [st['S'].data_ptr() + j * npad * 4 for j in range(self.m)]
            st['Y_ptr'] = [st['Y'].data_ptr() + j * npad * 4 for j in range(self.m)]
            self.state[k] = st
        return st

    @torch.no_grad()
    def step(self, vol, loss, loss_dev=None, loss_summed=False):
        """One L-BFGS step.  loss: the host value, or None with loss_dev (f64 device scalar),
        all-reduced with the dot vector (loss_summed: the ranks' values add up, else every rank
        holds the same value) and read with the first Armijo probes; returns the loss value (and
        skips the update when it is exactly 0, the converged case: the history, ring and Gram have
        then already taken this step's pair, so the caller stops iterating, optimize.py:305-307).  The recursion runs on the
        device (tvam_lbfgs_coef), so the history pass, the direction and its render follow each
        other on the stream: one host read per step (the probes), none before the render."""
        from . import _abi
        lib = self._lib()
        search = {}
        gdz_dev = []
        loss_cell = None
        for k, p in self.variables.items():
            st = self._st(k, p)
            pf = _aligned(p.detach().reshape(-1))
            g = _aligned(p.grad.detach().reshape(-1).contiguous())
            n = st['n']
            stream = self._stream(pf.device)
            new = st['t'] > 0
            if new and len(st['slots']) == self.m:  # evict the oldest pair (lbfgs.py:214-217)
                st['free'].append(st['slots'].pop(0))
            kept = list(st['slots'])
            h = len(kept)
            S_ptrs = (ctypes.c_void_p * max(h, 1))(*[st['S_ptr'][j] for j in kept])
            Y_ptrs = (ctypes.c_void_p * max(h, 1))(*[st['Y_ptr'][j] for j in kept])
            slot = st['free'][0] if new else None
            # the last update already wrote this pair's s = p - p_old into its slot (s_out of
            # tvam_axpy_clamp_dev) when p is still that update's output and p_old its input, unchanged
            sp, st['s_pre'] = st.get('s_pre'), None
            spre = (new and sp is not None and sp['slot'] == slot and sp['out'].data_ptr() == pf.data_ptr()
                    and sp['out']._version == sp['out_v'] and pf._version == sp['out_v']
                    and sp['p'] is st['p_old'] and st['p_old']._version == sp['p_v'])
            _abi.check(lib.tvam_lbfgs_history(
                n, pf.data_ptr() if new and not spre else None,
                st['p_old'].data_ptr() if new and not spre else None, g.data_ptr(),
                st['g_old'].data_ptr() if new else None, h, S_ptrs, Y_ptrs,
                st['S_ptr'][slot] if new else None, st['Y_ptr'][slot] if new else None,
                st['work'].data_ptr(), st['dots'].data_ptr(), stream))
            nd = 5 * (h + 1) + 1 if new else 2 * h + 1
            dots = st['dots'][:nd]
            with_loss = loss_dev is not None and loss is None and loss_cell is None
            if with_loss:
                dots = torch.cat([dots, loss_dev.reshape(1).to(torch.float64)])
            if self.allreduce is not None:
                dots = self.allreduce(dots.clone())
            if with_loss:
                loss_cell = dots[nd:nd + 1]
            if new:
                st['free'].pop(0)
                st['slots'].append(slot)
            order = st['slots']
            H = len(order)
            st['p_old'], st['g_old'] = pf, g
            st['t'] += 1
            # two-loop recursion on the Gram entries (lbfgs.py:221-243), on the device
            gdz = torch.empty(1, dtype=torch.float64, device=pf.device)
            order_c = (ctypes.c_int32 * max(H, 1))(*order)
            _abi.check(lib.tvam_lbfgs_coef(H, int(new), int(st['t'] == 1), order_c, dots.data_ptr(),
                                           st['gram'].data_ptr(), st['coef'].data_ptr(), gdz.data_ptr(), stream))
            d = torch.empty_like(g)
            S2 = (ctypes.c_void_p * max(H, 1))(*[st['S_ptr'][j] for j in order])
            Y2 = (ctypes.c_void_p * max(H, 1))(*[st['Y_ptr'][j] for j in order])
            _abi.check(lib.tvam_lbfgs_direction_dev(n, g.data_ptr(), H, S2, Y2, st['coef'].data_ptr(), d.data_ptr(),
                                                    stream))
            search[k] = d
            gdz_dev.append(gdz)

        def host_scalars(extra=None):
            """(loss, g.d summed over the variables[, extra values]) in one host read."""
            parts = ([loss_cell] if loss_cell is not None else []) + gdz_dev + ([extra] if extra is not None else [])
            v = torch.cat([t.reshape(-1).to(torch.float64) for t in parts]).cpu().tolist()
            lv = loss
            if loss_cell is not None:
                lv = v.pop(0)
                if self.allreduce is not None and not loss_summed:
                    import torch.distributed as _d
                    lv = lv / _d.get_world_size()
            gdz_total = 0.0
            for _ in gdz_dev:
                gdz_total += v.pop(0)
            return float(lv), gdz_total, v

        c1 = 1e-4
        params = {k: search[k].reshape(self.variables[k].shape) for k in self.variables}
        dvol = self.render_fn(params)
        key = 'projector.active_data' if 'projector.active_data' in params else next(iter(params))
        alpha = 1.0
        steps = 0
        lo = -float('inf') if self.clamp_min is None else float(self.clamp_min)
        spec = None  # (update, its step size on the device) launched behind the first probes
        if self.loss_steps is not None and self.search_it > 0:
            # the same backtracking sequence (alpha = 1, 1/2, ...; first Armijo pass wins), its
            # probes evaluated probe_batch at a time: one loss pass and one host read per batch
            # (the first read also carries the loss and g.d)
            done = False
            first = True
            while steps < self.search_it and not done:
                nb = min(self.probe_batch, self.search_it - steps)
                alphas = [alpha * 0.5 ** j for j in range(nb)]
                fd = self.loss_steps(vol, dvol, alphas, params[key])
                if first:
                    if self.speculate and len(self.variables) == 1 and fd.is_cuda and fd.dtype == torch.float64:
                        spec, loss_v, gdz_total, fv = self._speculative_update(fd, nb, c1, loss, loss_cell, gdz_dev[0],
                                                                               loss_summed, search, lo)
                    else:
                        loss_v, gdz_total, fv = host_scalars(fd)
                    first = False
                    if loss_cell is not None and loss_v == 0.0:  # converged (optimize.py:305-307): no update
                        return loss_v
                else:
                    fv = fd.cpu().tolist()
                for a, f_new in zip(alphas, fv):
                    steps += 1
                    alpha = a
                    if f_new <= loss_v + c1 * a * gdz_total:
                        done = True
                        break
                if not done:
                    alpha *= 0.5
        else:
            loss_v, gdz_total, _ = host_scalars()
            if loss_cell is not None and loss_v == 0.0:
                return loss_v
            for _ in range(self.search_it):
                steps += 1
                if self.loss_step is not None:
                    f_new = self.loss_step(vol, dvol, alpha, params[key])
                else:
                    f_new = self.loss_fn(vol + alpha * dvol, params[key])
                if float(f_new) <= loss_v + c1 * alpha * gdz_total:
                    break
                alpha *= 0.5
        self.last_alpha = alpha
        self.last_search_steps = steps

        if spec is not None and steps <= self.probe_batch and alpha == spec[1]:
            # the device picked the same step size in the same f64 arithmetic: its update stands (and
            # the s = p_new - p it wrote into the next pair's slot)
            (k, p), = self.variables.items()
            self.variables[k] = spec[0].reshape(p.shape).requires_grad_(True)
            if spec[2] is not None:
                self.state[k]['s_pre'] = spec[2]
            return loss_v
        for k, p in self.variables.items():
            pf = _aligned(p.detach().reshape(-1))
            out = torch.empty_like(pf)
            _abi.check(lib.tvam_axpy_clamp(pf.numel(), pf.data_ptr(), float(alpha), search[k].data_ptr(), lo,
                                           out.data_ptr(), self._stream(pf.device)))
            self.variables[k] = out.reshape(p.shape).requires_grad_(True)
        return loss_v
