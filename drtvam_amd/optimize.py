"""Pattern optimisation driver (mirror of drtvam/optimize.py).

``load_scene(config)`` assembles the scene dictionary exactly as
optimize.py:15-79 (vial, projector, sensor with scalex/y/z, target transform).
``TvamProblem`` holds everything one optimizer iteration touches and
``TvamProblem.iteration(i)`` is the loop body of optimize.py:287-323:

    forward render (seed=i) -> loss (+ dL/dD) -> host sync of the loss value
    -> adjoint render -> LinearLBFGS.step (1 more forward render + Armijo)
    -> clamp patterns at 0

With ThresholdedLoss on a binary target the loss, its gradient and every
Armijo probe run in the fused HIP loss kernel; other losses go through torch
autograd with the same render op.  Under torch.distributed the projector
angles are sharded across ranks: each rank renders its angles, the partial
dose is all-reduced (RCCL), the adjoint is rank-local and L-BFGS dots are
all-reduced scalars.
"""
from __future__ import annotations

import argparse
import ctypes
import math
import gc
import json
import os
import time
from typing import Optional

import numpy as np
import torch

from .engine import derive_seed_grad
from .geometry import geometries
from .integrators import VolumeIntegrator
from .lbfgs import DirectionPipeline, FusedLinearLBFGS, LinearLBFGS
from .loss import losses, ThresholdedLoss
from .scene import load_dict
from .utils import discretize, analytic_target, mesh_bbox, target_transform, save_vol, save_img


def load_scene(config):
    for key in ['target', 'vial', 'projector', 'sensor']:
        if key not in config:
            raise ValueError(f"Missing field '{key}' in the configuration file.")
    if 'type' not in config['vial']:
        raise ValueError("The vial geometry must have a 'type' field.")
    if config['vial']['type'] not in geometries.keys():
        raise ValueError(f"Unknown vial geometry: '{config['vial']['type']}'")
    vial = geometries[config['vial']['type']](config['vial'])

    tgt = dict(config['target'])
    if 'filename' not in tgt and 'analytic' not in tgt:
        raise ValueError("Missing field 'filename' for the target shape.")
    target = {'type': 'analytic', 'kind': tgt.get('analytic')}
    if 'filename' in tgt:
        bmin, bmax = mesh_bbox(tgt['filename'])
        center = (tgt.get('box_center_x', 0.), tgt.get('box_center_y', 0.), tgt.get('box_center_z', 0.))
        target = {'type': os.path.splitext(tgt['filename'])[1][1:], 'filename': tgt['filename'],
                  'to_world': target_transform(bmin, bmax, tgt.get('size', 1.), center), 'bsdf': {'type': 'null'}}

    def sensor_dict(sd):
        sd = dict(sd)
        sx, sy, sz = sd.pop('scalex', 1.), sd.pop('scaley', 1.), sd.pop('scalez', 1.)
        sd['to_world'] = np.diag([sx, sy, sz, 1.0])
        return sd

    scene_dict = {
        'type': 'scene',
        'projector': dict(config['projector']),
        'sensor': sensor_dict(config['sensor']),
        'target': target,
        '_container': vial,
    } | vial.to_dict()
    if 'final_sensor' in config:
        scene_dict['final_sensor'] = sensor_dict(config['final_sensor'])
    return scene_dict


def angle_shard(n_angles: int, rank: int, world: int):
    """Contiguous angle block [a0, a1) of `rank`."""
    return (n_angles * rank) // world, (n_angles * (rank + 1)) // world


# Relative cost of a film slice in a slab-sharded iteration: every slice costs its forward, vector
# and base adjoint work (1), and the adjoint marches a (45 x 45 tile, slice chunk) only where the
# thresholded loss's gradient is nonzero -- near convergence, the tiles that hold target voxels:
# + SLAB_TARGET_COST x the slice's fraction of such tiles.  From the round-5 8-rank emulation of
# config 2 (profiles/r05/final/emulate_slab.jsonl): slab 0 (10 of 50 slices in the box target) ran
# its adjoint in 0.206 ms, slab 3 (50 of 50) in 0.458 ms, i.e. 0.0063 ms more per target slice on
# a per-slice iteration cost of ~0.016 ms.
SLAB_TARGET_COST = 0.4
SLAB_TILE = 45


def slab_costs(target, tile=SLAB_TILE, gamma=SLAB_TARGET_COST):
    """Per-slice cost weights of a slab split from the target [Z, Y, X(, C)] (CPU tensor)."""
    t = torch.as_tensor(target)
    if t.dim() == 4:
        t = t[..., 0]
    occ = (t > 0).to(torch.float32)
    Z, Y, X = occ.shape
    py, px = (-Y) % tile, (-X) % tile
    occ = torch.nn.functional.pad(occ, (0, px, 0, py))
    tiles = occ.reshape(Z, (Y + py) // tile, tile, (X + px) // tile, tile).amax(dim=(2, 4))
    frac = tiles.reshape(Z, -1).mean(dim=1)
    return (1.0 + gamma * frac).double().numpy()


def balanced_slabs(costs, world):
    """Contiguous slabs [z0, z1) of the slices, one per rank, whose largest summed cost is least
    (binary search on the bound, greedy fill; every slab keeps at least one slice)."""
    n = len(costs)
    if world >= n:
        return [(min(k, n), min(k + 1, n)) for k in range(world)]
    pre = np.concatenate([[0.0], np.cumsum(costs)])

    def cut(bound):
        edges, z = [0], 0
        for k in range(world - 1):
            left = world - 1 - k  # slabs after this one, each needing a slice
            hi = n - left
            j = z + 1
            while j < hi and pre[j + 1] - pre[z] <= bound:
                j += 1
            edges.append(j)
            z = j
        edges.append(n)
        return edges, max(pre[b] - pre[a] for a, b in zip(edges[:-1], edges[1:]))

    lo, hi = float(max(costs)), float(pre[-1])
    best = cut(hi)
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        e, m = cut(mid)
        if m <= mid + 1e-12:
            hi, best = mid, (e, m)
        else:
            lo = mid
    e = best[0]
    return [(e[k], e[k + 1]) for k in range(world)]


def _dist(always=False):
    """torch.distributed when a process group of more than one rank is up (or of any size with
    `always`: config 'collectives': 'always' runs the sharded loop's collectives at world size 1)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and (always or dist.get_world_size() > 1):
        return dist
    return None


class ShardedLoop:
    """The optimisation loop of one angle shard (optimize.py:287-323), independent of
    how the shard's forward / adjoint projections are computed.

    Subclasses provide ``forward_local(x, seed) -> partial dose`` (this rank's
    angles only) and ``adjoint_local(grad_vol, seed) -> dL/dx_local``; the loop
    all-reduces the dose (torch.distributed, RCCL on GPUs / gloo on CPU), keeps
    the adjoint rank-local and all-reduces every L-BFGS dot product.
    Required attributes: loss_fn, target, n_global, fused, grad_vol, x0.
    """

    dist = None
    progressive = False
    max_depth = 6
    fused_lbfgs = True
    dose_sharded = False  # z-slab sharding: each rank owns a slab of the dose (no dose all-reduce)
    n_vox = None          # voxels of the whole film (normalises a 'mean' loss on a slab)

    def forward_local(self, x, seed):
        raise NotImplementedError

    def adjoint_local(self, grad_vol, seed):
        raise NotImplementedError

    def on_progressive(self):
        pass

    # ---- distributed helpers ------------------------------------------------
    def allreduce_(self, t):
        if self.dist is not None:
            self.dist.all_reduce(t)
        return t

    def dot(self, a, b):
        return self.allreduce_(torch.dot(a, b))

    def sparsity(self, x):
        lf = self.loss_fn
        w = getattr(lf, 'weight_sparsity', 0)
        if not w:
            return None
        v = self.allreduce_((torch.abs(x.detach()) ** lf.M).sum(dtype=torch.float64) * w)
        return v / self.n_active_global() if lf.reduction_name == 'mean' else v

    def n_active_global(self):
        """Entries of projector.active_data (after filter_radon, the pixels that stayed active)."""
        return getattr(self, 'n_filtered', None) or self.n_global

    def sparsity_grad(self, x):
        lf = self.loss_fn
        w = getattr(lf, 'weight_sparsity', 0)
        if not w:
            return None
        g = w * lf.M * torch.abs(x.detach()) ** (lf.M - 1) * torch.sign(x.detach())
        return g / self.n_active_global() if lf.reduction_name == 'mean' else g

    # ---- projections ----------------------------------------------------------
    allreduce_chunks = 4  # angle shards: slice ranges whose dose all-reduce overlaps the next range's forward

    def forward_chunks(self):
        """Film slice ranges [(z0, z1), ...] of an overlapped forward + all-reduce, or None."""
        return None

    def forward_local_slices(self, x, seed, z0, z1, out):
        raise NotImplementedError

    def dose_buffer(self):
        raise NotImplementedError

    def direction_pipeline(self):
        """A DirectionPipeline (the iteration in slab bands, projections of one band overlapping the
        vector passes of the next), or None."""
        return None

    def forward(self, x, seed):
        """This rank's partial dose, all-reduced over the angle shards.  When the
        projection can render slice ranges, range k's all-reduce (async: RCCL runs it on its own
        stream) overlaps range k + 1's forward; the sum per voxel is the same."""
        if self.dose_sharded:
            return self.forward_local(x, seed)
        chunks = self.forward_chunks() if self.dist is not None else None
        if not chunks:
            return self.allreduce_(self.forward_local(x, seed))
        vol = self.dose_buffer()
        works = []
        for z0, z1 in chunks:
            self.forward_local_slices(x, seed, z0, z1, vol)
            works.append(self.dist.all_reduce(vol[z0:z1], async_op=True))
        for w in works:
            w.wait()
        return vol

    def adjoint(self, grad_vol, seed):
        return self.adjoint_local(grad_vol, seed)

    # ---- loss -------------------------------------------------------------------
    def loss_value_grad(self, vol, x, reduce=True):
        """(loss f64 device scalar, dL/dvol) — fused kernel or torch autograd.  The film
        term is summed over the slabs when the dose is sharded (reduce=False leaves this
        rank's slab term, for a caller that folds the sum into a later all-reduce); the
        sparsity term (loss.py:54-59) is added once, summed over the pattern shards."""
        s = self.sparsity(x)
        if self.fused:
            v = self.loss_fn.fused_value_grad(vol, self.target, None, self.grad_vol, count=self.n_vox)
            if self.dose_sharded and reduce:
                v = self.allreduce_(v)
            if s is not None and not reduce and self.dose_sharded and self.dist is not None:
                s = s / self.dist.get_world_size()  # summed again with the slab terms
            return (v if s is None else v + s), self.grad_vol
        vv = vol.detach().requires_grad_(True)
        with torch.enable_grad():
            l = self.loss_fn(vv, self.target, torch.zeros_like(x))
            l.backward()
        l = l.detach().to(torch.float64)
        if self.dose_sharded:
            l = self.allreduce_(l)
        return (l if s is None else l + s), vv.grad

    def loss_step(self, vol, dvol, alpha, patterns):
        s = self.sparsity(patterns)
        if self.fused:
            v = self.loss_fn.fused_value(vol, self.target, None, dvol, alpha, count=self.n_vox)
        else:
            v = self.loss_fn(vol + alpha * dvol, self.target, torch.zeros_like(patterns)).to(torch.float64)
        if self.dose_sharded:
            v = self.allreduce_(v)
        return v if s is None else v + s

    def loss_steps(self, vol, dvol, alphas, patterns):
        """loss_step for several step sizes at once (fused loss only): f64 device vector, one
        loss pass and, on a sharded dose, one all-reduce."""
        s = self.sparsity(patterns)
        v = self.loss_fn.fused_values(vol, self.target, None, dvol, alphas, count=self.n_vox)
        if self.dose_sharded:
            v = self.allreduce_(v)
        return v if s is None else v + s

    # ---- optimisation -------------------------------------------------------------
    def make_optimizer(self):
        key = 'projector.active_data'

        def render_fn(vars_):
            return self.forward(vars_[key], self._seed)

        dev = getattr(self, 'device', None) or self.x0.device
        if dev.type == 'cuda' and self.fused_lbfgs:
            # three fused HIP passes per step and one all-reduce of the dot vector
            opt = FusedLinearLBFGS(render_fn=render_fn, loss_fn=None, loss_step=self.loss_step,
                                   allreduce=self.allreduce_ if self.dist is not None else None, clamp_min=0.0,
                                   loss_steps=self.loss_steps if self.fused else None,
                                   pipeline=self.direction_pipeline())
        else:
            opt = LinearLBFGS(render_fn=render_fn, loss_fn=None, dot=self.dot, loss_step=self.loss_step)
        opt[key] = self.x0
        self.opt = opt
        return opt

    def iteration(self, i):
        """One optimizer iteration (optimize.py:292-320).  Returns the loss value."""
        if self.opt is None:
            self.make_optimizer()
        if self.progressive and i == 5:
            self.on_progressive()
        key = 'projector.active_data'
        self._seed = i
        x = self.opt[key]
        if isinstance(self.opt, FusedLinearLBFGS) and self.fused and self.opt.pipeline is not None:
            loss_v = self._iteration_pipelined(x, i)
            self.loss_hist.append(loss_v)
            return loss_v
        vol = self.forward(x, i)
        if isinstance(self.opt, FusedLinearLBFGS) and self.fused:
            # The loss value is read with the L-BFGS dot vector: the adjoint and the history
            # pass run first, and one collective + one host sync carry both (the reference
            # reads the loss right away, optimize.py:303; the value and the update agree).
            loss, gvol = self.loss_value_grad(vol, x, reduce=False)
            g = self.adjoint(gvol, i)
            sg = self.sparsity_grad(x)
            if sg is not None:
                g = g + sg
            x.grad = g
            loss_v = self.opt.step(vol, None, loss_dev=loss, loss_summed=self.dose_sharded)
            self.loss_hist.append(loss_v)
            return loss_v
        loss, gvol = self.loss_value_grad(vol, x)
        loss_v = float(loss)  # host sync, optimize.py:303
        self.loss_hist.append(loss_v)
        g = self.adjoint(gvol, i)
        sg = self.sparsity_grad(x)
        if sg is not None:
            g = g + sg
        x.grad = g
        if loss_v == 0.0:
            return loss_v
        self.opt.step(vol, loss_v)
        if getattr(self.opt, 'clamp_min', None) != 0.0:  # the fused optimizer clamps in its update pass
            with torch.no_grad():
                self.opt[key] = torch.clamp_min(self.opt[key].detach(), 0.0)
        return loss_v

    def _iteration_pipelined(self, x, i):
        """iteration() in slab bands (DirectionPipeline): the forward of band k on the current
        stream, its loss + dL/dvol on the side stream (hidden under band k + 1's forward), then band
        k's adjoint (tvam_adjoint_slices, its pattern rows) on the current stream while the side
        stream runs band k - 1's history pass; FusedLinearLBFGS.step_pipelined continues the same
        way through the direction, its render and the probes.  The same kernels per element as the
        unbanded iteration; the loss, the dots and the probes are summed over the bands."""
        pipe = self.opt.pipeline
        dev = self.device
        main = torch.cuda.current_stream(dev)
        side = pipe.side(dev)
        xd = x.detach().contiguous()
        vol = self.dose_buffer()
        loss_evs, loss_parts = [], []
        for r0, r1, z0, z1 in pipe.parts:
            pipe.render_part(xd, z0, z1, vol)
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                loss_parts.append(self.loss_fn.fused_value_grad(vol[z0:z1], self.target[z0:z1], None,
                                                                self.grad_vol[z0:z1], count=self.n_vox))
                evl = torch.cuda.Event()
                evl.record(side)
            loss_evs.append(evl)
        # the gradient zeroed once (one contiguous fill: tvam_adjoint_slices' own zeroing of a row
        # band is a strided 2-D fill over every angle, 6x slower), then every band adds into it
        # (an empty row range: no zeroing)
        g = torch.zeros(self.n_local, dtype=torch.float32, device=dev)
        grad_ready = []
        for (r0, r1, z0, z1), evl in zip(pipe.parts, loss_evs):
            main.wait_event(evl)
            self.proj.adjoint_slices(self.grad_vol, self.n_local, z0, z1, r0, r0, g)
            ev = torch.cuda.Event()
            ev.record(main)
            grad_ready.append((ev, r0, r1))
        x.grad = g
        return self.opt.step_pipelined(vol, loss_parts, self.dose_sharded, grad_ready)

    def patterns_local(self):
        return self.opt['projector.active_data'].detach() if self.opt is not None else self.x0



def slab_bands(m, nz, n, zc, za, R):
    """[(row0, row1, z0, z1), ...] of a banded planar iteration, or None: about n film slice ranges
    with boundaries on whole forward (zc) / adjoint (za) slice chunks and 64-slice bin blocks, each
    with the one contiguous band of DMD rows whose rays lie in it (m = each crop row's film slice,
    -1: misses the grid; rows may run top-down or bottom-up); the bands, extended over the unmapped
    rows between them, tile [0, R)."""
    blk = 64 * zc // math.gcd(64, zc)
    blk = blk * za // math.gcd(blk, za)
    cuts = sorted({min(nz, max(0, int(round(j * nz / n / blk)) * blk)) for j in range(1, n)} - {0, nz})
    edges = [0] + cuts + [nz]
    ranges = list(zip(edges[:-1], edges[1:]))
    if len(ranges) <= 1:
        return None
    m = np.asarray(m)
    mapped = m >= 0
    bands = []
    for z0, z1 in ranges:
        rows = np.nonzero(mapped & (m >= z0) & (m < z1))[0]
        if not rows.size:
            return None
        lo, hi = int(rows.min()), int(rows.max()) + 1
        if not np.all(((m[lo:hi] >= z0) & (m[lo:hi] < z1)) | ~mapped[lo:hi]):
            return None
        bands.append((lo, hi))
    order = sorted(range(len(ranges)), key=lambda q: bands[q][0])
    ext = {}
    for j, q in enumerate(order):
        lo = 0 if j == 0 else bands[q][0]
        hi = R if j == len(order) - 1 else bands[order[j + 1]][0]
        if hi < bands[q][1]:
            return None  # overlapping bands
        ext[q] = (lo, hi)
    return [(ext[q][0], ext[q][1], z0, z1) for q, (z0, z1) in enumerate(ranges)]

class TvamProblem(ShardedLoop):
    """Scene + target + loss + optimizer state of one optimisation run (one rank's angle shard)."""

    def __init__(self, config, device=None, target=None, rank=None, world_size=None, filter_pixels=True):
        self.config = config
        self.dist = _dist(always=config.get('collectives') == 'always')
        self.rank = rank if rank is not None else (self.dist.get_rank() if self.dist else 0)
        self.world = world_size if world_size is not None else (self.dist.get_world_size() if self.dist else 1)
        dev = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        proj_cfg = dict(config['projector'])
        proj_cfg['device'] = dev
        cfg = dict(config)
        cfg['projector'] = proj_cfg
        self.scene_dict = load_scene(cfg)
        self.scene = load_dict(self.scene_dict)
        self.sensor = self.scene.sensor_by_id('sensor')
        ids = self.scene.sensor_ids()
        self.final_sensor = self.scene.sensor_by_id('final_sensor') if 'final_sensor' in ids else self.sensor
        if self.final_sensor.film().surface_aware:
            raise ValueError("The final sensor is used to generate visualizations and metrics of the final simulated print. Therefore, it must not be surface-aware. If you are using the surface-aware discretization for optimization, please specify another sensor called 'final_sensor' in the configuration file.")
        self.device = dev

        self.spp = config.get('spp', 4)
        self.spp_ref = config.get('spp_ref', 16)
        self.spp_grad = config.get('spp_grad', self.spp)
        self.max_depth = config.get('max_depth', 6)
        self.rr_depth = config.get('rr_depth', 6)
        self.time = config.get('time', 1.)
        self.progressive = config.get('progressive', False)
        self.transmission_only = config.get('transmission_only', True)
        self.regular_sampling = config.get('regular_sampling', False)
        self.n_steps = config.get('n_steps', 40)

        lcfg = dict(config.get('loss', {'type': 'threshold'}))
        ltype = lcfg.pop('type', 'threshold')
        if ltype not in losses:
            raise ValueError(f"Unknown loss type: '{ltype}'. Available losses are: {list(losses.keys())}")
        self.loss_fn = losses[ltype](lcfg)
        lf = self.loss_fn
        fusable = (isinstance(lf, ThresholdedLoss) and dev.type == 'cuda' and float(lf.K).is_integer()
                   and 1 <= int(lf.K) <= 16)

        # Sharding.  'angle': contiguous angle blocks, the
        # partial doses are all-reduced.  'slab': planar rays (regular sampling)
        # never leave their z-slice, so rank k owns a slab of film slices and the
        # band of DMD rows whose rays lie in it, for every angle: no dose
        # communication at all (only scalar loss / dot all-reduces).
        A = self.scene.projector.n_patterns
        shard = config.get('shard', 'auto')
        if shard not in ('auto', 'angle', 'slab'):
            raise ValueError(f"Unknown shard mode '{shard}' (auto, angle, slab)")
        base = {'max_depth': 3 if self.progressive else self.max_depth, 'rr_depth': self.rr_depth,
                'print_time': self.time, 'transmission_only': self.transmission_only,
                'regular_sampling': self.regular_sampling, 'tile': config.get('tile', 0),
                'flags': config.get('flags', 0)}
        p = self.scene.projector
        if not p.dense:
            raise NotImplementedError("sharded optimisation needs the dense active set")
        self.crop_x, self.crop_y = p.crop[0], p.crop[1]
        full_desc = VolumeIntegrator(base).desc(self.scene, self.sensor)
        self.res_z = int(full_desc.film_res[2])
        if 'flags' not in config and full_desc.albedo != 0.0:
            # every path marched, as the reference marches every active pixel (projector.py:66-70,
            # common.py:81-82): a scattering scene's paths then do not depend on the pattern, and
            # the line-search forward is served from the forward bin cache (lbfgs.py:240-249)
            from ._abi import FLAG_NO_ZERO_SKIP
            base['flags'] = int(base['flags']) | FLAG_NO_ZERO_SKIP
        self.surface_aware = bool(self.sensor.film().surface_aware)
        if target is None:
            if self.surface_aware:  # fractional inside / outside volumes (optimize.py:131-134)
                target = self.sensor.compute_volume(self.scene).cpu()
            elif 'filename' in config['target']:
                target = discretize(self.scene, sensor=self.sensor)
            else:
                target = analytic_target(self.sensor.resolution(), self.sensor.bbox_min, self.sensor.bbox_max,
                                         config['target'].get('analytic', 'box_hole'))
        self.target_full = target.to(dtype=torch.float32)
        # scattered paths leave their slice; surface-aware films run the per-path kernels
        planar = self.regular_sampling and full_desc.albedo == 0.0 and not self.surface_aware
        if shard == 'slab' and not (planar and fusable):
            raise ValueError("z-slab sharding needs regular sampling, a non-scattering medium and the fused "
                             "thresholded loss")
        self.shard = 'slab' if (shard == 'slab' or (shard == 'auto' and self.world > 1 and planar
                                                     and fusable)) else 'angle'
        self.n_vox = int(full_desc.film_res[0]) * int(full_desc.film_res[1]) * self.res_z
        if self.shard == 'slab':
            self.a0, self.a1 = 0, A
            # slabs of equal cost (slab_costs), the same on every rank
            self.slabs = balanced_slabs(slab_costs(self.target_full.cpu()), self.world)
            self.z0, self.z1 = self.slabs[self.rank]
            self.r0, self.r1 = self._row_band(full_desc)
            shard_props = {'angle_range': (0, A), 'row_band': (self.r0, self.r1), 'slab': (self.z0, self.z1)}
            self.dose_sharded = True
        else:
            self.a0, self.a1 = angle_shard(A, self.rank, self.world)
            self.z0, self.z1, self.r0, self.r1 = 0, self.res_z, 0, self.crop_y
            shard_props = {'angle_range': (self.a0, self.a1)}
        self.base_props = dict(base)
        iprops = base | shard_props
        self.integrator = VolumeIntegrator(iprops)
        self.final_integrator = VolumeIntegrator(iprops | {'max_depth': config.get('max_depth_ref', 16),
                                                           'rr_depth': config.get('rr_depth_ref', 8)})

        self.target = self.target_full[self.z0:self.z1].to(device=dev).contiguous()

        # this rank's part of projector.active_data (dense crop order [angle][row][col])
        per_angle = self.crop_x * self.crop_y
        self.n_global = A * per_angle
        self.n_local = (self.a1 - self.a0) * (self.r1 - self.r0) * self.crop_x
        self.x0 = self.local_from_global(p.active_data)
        # the dense crop order unless filter_radon compacts the set; the ray weight divides by
        # the whole (all ranks') active set size, as the unsharded reference does
        self.active_pixels = None
        self.active_dense = None
        self.active_set = (0, self.n_global)
        self.proj = self._active_projection(self.integrator, self.sensor)
        if config.get('filter_radon', False) and filter_pixels:
            self._filter_radon(config)
        self.fused = fusable and self.target.shape[-1] == 1
        self.grad_vol = torch.empty(self.proj.film_shape, dtype=torch.float32, device=dev)
        self.opt = None
        self.loss_hist = []
        self.timing = []

    def _filter_radon(self, config):
        """Deactivate the pixels whose rays never cross the target inside the medium
        (optimize.py:143-163): the Radon integrator (max_depth 5, jittered, spp_filter_radon
        samples) on this rank's pixels, then the active set is compacted like the reference's
        dr.compress: projector.active_pixels holds only the surviving pixels (full-DMD indices
        in dense order), active_data is a zero vector of that length, and the forward, the
        adjoint and every L-BFGS vector run over the compacted set.  Sampler streams follow
        the position in the whole (all ranks') active set, as common.py:57-67 seeds them."""
        from .engine import Projection
        from .utils import target_triangles
        d = self.proj.desc.copy()
        d.regular_sampling = 0
        d.max_depth = 5
        d.flags |= 4  # TVAM_FLAG_NO_PLANAR: no planar tables needed for a setup pass
        radon = Projection(d, self.device).radon(target_triangles(self.scene), spp=config.get('spp_filter_radon', 4),
                                                 seed=0, max_depth=5)
        local = torch.nonzero(radon > 0).reshape(-1)  # dense indices of this rank's shard, ascending
        counts = [int(local.numel())]
        if self.dist is not None:
            counts = [None] * self.world
            self.dist.all_gather_object(counts, int(local.numel()))
        self.n_filtered = int(sum(counts))
        if self.n_filtered == 0:
            raise ValueError("No active pixels found in the Radon transform.")
        # full-DMD pixel index of each surviving dense entry [angle][crop row][crop col] of the plan
        pd = self.proj.desc
        cx, cy = int(pd.crop_x), int(pd.crop_y)
        al = local // (cx * cy)
        rem = local - al * (cx * cy)
        row = rem // cx
        col = rem - row * cx
        W, H = int(pd.res_x), int(pd.res_y)
        pix = (al + int(pd.angle_begin)) * (W * H) + (row + int(pd.crop_offset_y)) * W + col + int(pd.crop_offset_x)
        if pix.numel() and int(pix.max()) >= 2 ** 31:
            raise ValueError("filter_radon: DMD pixel index exceeds the int32 active_pixels range")
        self.active_pixels = pix.to(torch.int32).contiguous()
        self.active_dense = local  # scatter positions of the compacted vector in this rank's dense layout
        self.n_dense_local = self.n_local
        self.n_local = int(local.numel())
        # angle shards are contiguous blocks of the global dense order: this rank's first
        # active entry sits after every lower rank's (slab shards interleave, but run only
        # under regular sampling, where no sampler stream is drawn)
        self.active_set = (sum(counts[:self.rank]) if self.shard == 'angle' else 0, self.n_filtered)
        self.proj.set_active(*self.active_set)
        self.x0 = torch.zeros(self.n_local, dtype=torch.float32, device=self.device)

    def _row_band(self, desc):
        """Crop rows [r0, r1) whose rays lie in this rank's slab (rows outside the grid go to the
        outermost bands, so the bands tile all crop rows)."""
        from . import _abi
        m = np.empty(desc.crop_y, dtype=np.int32)
        _abi.check(_abi.load_library().tvam_row_slices(ctypes.byref(desc), m.ctypes.data_as(ctypes.c_void_p)))
        bands = []
        for k in range(self.world):
            z0, z1 = self.slabs[k]
            rows = np.nonzero((m >= z0) & (m < z1))[0]
            bands.append((int(rows.min()), int(rows.max()) + 1) if rows.size else None)
            if rows.size and not np.all((m[rows.min():rows.max() + 1] >= z0) & (m[rows.min():rows.max() + 1] < z1)
                                        | (m[rows.min():rows.max() + 1] < 0)):
                raise ValueError("z-slab sharding: the rows of a slab are not contiguous")
        order = sorted((b[0], k) for k, b in enumerate(bands) if b is not None)
        if not order:
            raise ValueError("z-slab sharding: no DMD row reaches the grid")
        edges = {}
        for i, (_, k) in enumerate(order):  # extend bands over unmapped rows: [start of band, start of next)
            lo = 0 if i == 0 else bands[k][0]
            hi = desc.crop_y if i == len(order) - 1 else bands[order[i + 1][1]][0]
            edges[k] = (lo, hi)
        return edges.get(self.rank, (0, 0))

    def local_from_global(self, full):
        """This rank's part (angle block or row band) of a global dense pattern vector."""
        full = torch.as_tensor(full).reshape(-1, self.crop_y, self.crop_x)
        return full[self.a0:self.a1, self.r0:self.r1, :].reshape(-1).to(self.device).contiguous()

    def dense_local(self, local):
        """This rank's patterns in its dense layout (zeros at the pixels filter_radon disabled:
        projector.patterns(), projector.py:125-129)."""
        if self.active_dense is None:
            return local
        full = torch.zeros(self.n_dense_local, dtype=local.dtype, device=local.device)
        full[self.active_dense] = local
        return full

    def gather_patterns(self, local):
        """The global dense pattern vector (every rank), from the ranks' parts."""
        local = self.dense_local(local)
        if self.dist is None:
            return local
        A = self.scene.projector.n_patterns
        shapes = [None] * self.world
        self.dist.all_gather_object(shapes, (self.a0, self.a1, self.r0, self.r1))
        m = max((a1 - a0) * (r1 - r0) * self.crop_x for a0, a1, r0, r1 in shapes)
        buf = torch.zeros(m, dtype=local.dtype, device=local.device)
        buf[:local.numel()] = local
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        self.dist.all_gather(parts, buf)
        full = torch.zeros((A, self.crop_y, self.crop_x), dtype=local.dtype, device=local.device)
        for (a0, a1, r0, r1), part in zip(shapes, parts):
            n = (a1 - a0) * (r1 - r0) * self.crop_x
            full[a0:a1, r0:r1, :] = part[:n].reshape(a1 - a0, r1 - r0, self.crop_x)
        return full.reshape(-1)

    def gather_dose(self, vol):
        """The whole film from the ranks' slabs (slab sharding; the angle mode all-reduces)."""
        if self.dist is None or not self.dose_sharded:
            return vol
        slabs = [None] * self.world
        self.dist.all_gather_object(slabs, (self.z0, self.z1))
        m = max(z1 - z0 for z0, z1 in slabs)
        buf = torch.zeros((m,) + tuple(vol.shape[1:]), dtype=vol.dtype, device=vol.device)
        buf[:vol.shape[0]] = vol
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        self.dist.all_gather(parts, buf)
        return torch.cat([part[:z1 - z0] for (z0, z1), part in zip(slabs, parts)])

    def forward_local(self, x, seed):
        return self.proj.forward(x.detach().contiguous(), self.active_pixels, self.spp, seed)

    def forward_chunks(self):
        n = int(self.config.get('allreduce_chunks', self.allreduce_chunks))
        zc = self.proj.fwd_chunk
        nz = self.proj.film_shape[0]
        if n <= 1 or zc <= 0 or nz < 2 * zc:
            return None
        step = -(-(-(-nz // n)) // zc) * zc  # ceil(nz / n) rounded up to the forward's slice chunk
        return [(z0, min(nz, z0 + step)) for z0 in range(0, nz, step)]

    def forward_local_slices(self, x, seed, z0, z1, out):
        return self.proj.forward_slices(x.detach().contiguous(), self.active_pixels, self.spp, seed, z0, z1, out)

    def dose_buffer(self):
        return torch.empty(self.proj.film_shape, dtype=torch.float32, device=self.device)

    # slab bands of a pipelined iteration (config 'direction_parts'; <= 1: off).  Off by default:
    # measured slower on config 2 (3 bands: 83.1 / 83.7 -> 75.8 / 75.9 it/s, profiles/r04/ab12/), the
    # banded launches' tails and the concurrent vector passes cost the LDS-bound projections more
    # than the passes they hide
    direction_parts = 1

    def direction_pipeline(self):
        """Row bands of the dense local patterns whose film slices tile the plan's film in ranges
        of whole 64-slice blocks (the slice-binned forward bins per 64 slices): band k's render
        needs only band k's rows.  Planar voxel-driven forwards of a dense set on one rank or one
        z-slab (the angle-sharded forward all-reduces its ranges instead)."""
        from . import _abi
        n = int(self.config.get('direction_parts', self.direction_parts))
        zc, za = self.proj.fwd_chunk, self.proj.adj_chunk
        nz = self.proj.film_shape[0]
        if (n <= 1 or zc <= 1 or za <= 0 or self.active_pixels is not None or not self.fused or
                getattr(self.loss_fn, 'weight_sparsity', 0) or (self.dist is not None and not self.dose_sharded)
                or self.device.type != 'cuda' or self.proj.film_shape[-1] != 1):
            return None
        desc = self.proj.desc
        m = np.empty(desc.crop_y, dtype=np.int32)
        _abi.check(_abi.load_library().tvam_row_slices(ctypes.byref(desc), m.ctypes.data_as(ctypes.c_void_p)))
        m = np.where(m >= 0, m - int(desc.slab_begin), -1)  # this plan's film slices
        R, C = int(desc.crop_y), int(desc.crop_x)
        parts = slab_bands(m, nz, n, zc, za, R) if C % 4 == 0 else None
        if parts is None:
            return None
        nseg = self.n_local // (R * C)
        if nseg * R * C != self.n_local:
            return None

        def render_part(d, z0, z1, out):
            self.proj.forward_slices(d, None, self.spp, self._seed, z0, z1, out)

        def probe_part(vol, dvol, alphas, z0, z1):
            return self.loss_fn.fused_values(vol[z0:z1], self.target[z0:z1], None, dvol[z0:z1], alphas,
                                             count=self.n_vox)

        def reduce(t):
            return self.allreduce_(t) if self.dose_sharded else t

        return DirectionPipeline(nseg, R, C, parts, render_part, probe_part, reduce, self.dose_buffer)

    def adjoint_local(self, grad_vol, seed):
        return self.proj.adjoint(grad_vol, self.n_local, self.active_pixels, self.spp_grad, derive_seed_grad(seed))

    def _active_projection(self, integrator, sensor):
        proj = integrator.projection(self.scene, sensor)
        proj.set_active(*self.active_set)
        return proj

    def on_progressive(self):
        self.integrator.max_depth = self.max_depth
        self.proj = self._active_projection(self.integrator, self.sensor)
        if getattr(self.opt, 'pipeline', None) is not None:
            # the new plan may chunk its slices differently: re-derive the slab bands (or run the
            # unbanded iteration when they no longer tile its film)
            self.opt.pipeline = self.direction_pipeline()

    def final_render(self, spp=None):
        proj = self._active_projection(self.final_integrator, self.final_sensor)
        vol = proj.forward(self.patterns_local().contiguous(), self.active_pixels, spp or self.spp_ref, 0)
        return self.gather_dose(vol) if self.dose_sharded else self.allreduce_(vol)


def optimize(config, patterns_fwd=None, device=None):
    """Optimise the patterns (optimize.py:81-368).  Returns the final dose volume."""
    prob = TvamProblem(config, device=device, filter_pixels=patterns_fwd is None)
    output = config.get('output', '.')
    os.makedirs(output, exist_ok=True)
    if prob.rank == 0:
        tgt = prob.target_full.cpu().numpy()
        if prob.surface_aware:
            save_vol(tgt[..., 0, None], os.path.join(output, "target_in.exr"))
            save_vol(tgt[..., 1, None], os.path.join(output, "target_out.exr"))
        else:
            save_vol(tgt, os.path.join(output, "target.exr"))
        np.save(os.path.join(output, "target.npy"), tgt)
    p = prob.scene.projector
    if patterns_fwd is not None:
        print("Using provided patterns for forward mode.")
        pf = np.asarray(patterns_fwd, dtype=np.float32)
        if pf.ndim == 3 and tuple(pf.shape[1:]) == (p.res[1], p.res[0]) and tuple(p.crop) != tuple(p.res):
            ox, oy = p.crop_offset  # full-DMD patterns (patterns.npz): keep the crop
            pf = pf[:, oy:oy + p.crop[1], ox:ox + p.crop[0]]
        prob.x0 = prob.local_from_global(pf.reshape(-1))
    elif "psf_analysis" in config:
        return psf_analysis(prob, config, output)
    else:
        print("Optimizing patterns...")
        # the scene, plan and tensors live for the whole loop: keep them out of the cyclic GC's
        # generations (a full collection mid-loop stalls the host between two launches); unfrozen
        # afterwards, so the problem's prob <-> opt cycle and its plans are collected on return
        gc.collect()
        gc.freeze()
        try:
            for i in range(prob.n_steps):
                t0 = time.perf_counter()
                loss = prob.iteration(i)
                torch.cuda.synchronize()
                prob.timing.append(time.perf_counter() - t0)
                if loss == 0.0:
                    print("Converged")
                    break
        finally:
            gc.unfreeze()
    print("Rendering final state...")
    vol_final = prob.final_render()
    pats = prob.gather_patterns(prob.patterns_local().float())
    if prob.rank == 0:
        crop = pats.cpu().numpy().reshape(-1, p.crop[1], p.crop[0])
        _save_outputs(output, prob, vol_final, full_dmd(p, crop))
        if prob.surface_aware:  # the binary target on the final sensor's grid (optimize.py:355-360)
            tb = discretize(prob.scene, sensor=prob.final_sensor).numpy()
            np.save(os.path.join(output, "target_binary.npy"), tb)
            save_vol(tb, os.path.join(output, "target_binary.exr"))
    return vol_final


def full_dmd(p, crop):
    """The full DMD stack [n, res_y, res_x] of crop-order patterns (projector.patterns(),
    projector.py:125-129: zeros outside the crop)."""
    full = np.zeros((crop.shape[0], p.res[1], p.res[0]), dtype=np.float32)
    ox, oy = p.crop_offset
    full[:, oy:oy + p.crop[1], ox:ox + p.crop[0]] = crop
    return full


def _save_outputs(output, prob, vol_final, full):
    """final.npy / final.exr, loss / timing, patterns/NNNN.exr and patterns(.npz, _normalized_uint8.npz)
    (optimize.py:330-353)."""
    vf = vol_final.cpu().numpy()
    np.save(os.path.join(output, "final.npy"), vf)
    save_vol(vf, os.path.join(output, "final.exr"))
    np.save(os.path.join(output, "loss.npy"), np.asarray(prob.loss_hist))
    np.save(os.path.join(output, "timing.npy"), np.asarray(prob.timing))
    print("Saving images...")
    os.makedirs(os.path.join(output, "patterns"), exist_ok=True)
    for i in range(full.shape[0]):
        save_img(full[i], os.path.join(output, "patterns", f"{i:04d}.exr"))
    np.savez_compressed(os.path.join(output, "patterns.npz"), patterns=full)
    mx = float(full.max()) if full.size else 0.0
    if mx > 0:
        np.savez_compressed(os.path.join(output, "patterns_normalized_uint8.npz"),
                            patterns=(full / mx * 255).astype(np.uint8))
        print("Pattern efficiency {:.4f}".format(float(np.sum(full / mx / full.size))))


def psf_analysis(prob, config, output):
    """Dose of single DMD pixels (optimize.py:245-283): the active set is the listed pixels
    (index_pattern, y, x) on the full DMD with their intensities; one render with the
    reference integrator settings on the final sensor."""
    p = prob.scene.projector
    xres, yres = config["projector"]["resx"], config["projector"]["resy"]
    entries = config["psf_analysis"]
    print("\nPSF analysis enabled.")
    print("Number of traced pixels:", len(entries))
    pix = np.zeros(len(entries), dtype=np.int64)
    data = np.ones(len(entries), dtype=np.float32)
    for i, e in enumerate(entries):
        assert e["x"] < xres, "Invalid entry in psf_analysis: x out of bounds. Please check the configuration file."
        assert e["y"] < yres, "Invalid entry in psf_analysis: y out of bounds. Please check the configuration file."
        assert e["index_pattern"] < config["projector"]["n_patterns"], \
            "Invalid entry in psf_analysis: index_pattern out of bounds. Please check the configuration file."
        pix[i] = xres * yres * e["index_pattern"] + xres * e["y"] + e["x"]
        data[i] *= e["intensity"]
    if prob.world > 1:
        raise NotImplementedError("psf_analysis runs on one rank")
    integ = VolumeIntegrator(prob.base_props | {'max_depth': config.get('max_depth_ref', 16),
                                                'rr_depth': config.get('rr_depth_ref', 8)})
    proj = integ.projection(prob.scene, prob.final_sensor)
    dev = prob.device
    print("Rendering final state...")
    vol = proj.forward(torch.as_tensor(data, device=dev), torch.as_tensor(pix.astype(np.int32), device=dev),
                       prob.spp_ref, 0)
    full = np.zeros((p.n_patterns, yres, xres), dtype=np.float32)
    full.reshape(-1)[pix] = data
    _save_outputs(output, prob, vol, full)
    return vol


class OverrideAction(argparse.Action):
    def __init__(self, option_strings, dest, nargs=None, **kwargs):
        super().__init__(option_strings, dest, **kwargs)
        self.overrides = {}

    def __call__(self, parser, namespace, values, option_string=None):
        try:
            key, value = values.split('=')
        except ValueError:
            raise ValueError("Invalid parameter override. Use the format '-D key=value'")
        try:
            value = int(value)
        except ValueError:
            try:
                value = float(value)
            except ValueError:
                pass
        self.overrides[key] = value
        setattr(namespace, self.dest, self.overrides)


def apply_overrides(config, overrides):
    for key, value in (overrides or {}).items():
        key = key.split('.')
        tmp = config
        for k in key[:-1]:
            tmp = tmp[k]
        tmp[key[-1]] = value
    return config


def main(argv=None):
    parser = argparse.ArgumentParser("Optimize patterns for TVAM.")
    parser.add_argument("config", type=str, help="Path to the configuration file")
    parser.add_argument("-D", dest="overrides", metavar="key=value", action=OverrideAction,
                        help="Override/Add a parameter in the configuration dictionary. Nested keys are separated by dots.")
    parser.add_argument("--backend", type=str, default="hip", choices=["hip", "cuda", "llvm"],
                        help="Kept for CLI compatibility; the engine always runs the HIP kernels.")
    parser.add_argument("--forward_mode", action="store_true", help="Just project the patterns without optimization.")
    parser.add_argument("--patterns", type=str, help="Path to the patterns file (a .npz file). Only used in forward mode.")
    args = parser.parse_args(argv)
    with open(args.config, 'r') as f:
        config = json.load(f)
    apply_overrides(config, args.overrides)
    if 'output' not in config:
        config['output'] = os.path.dirname(os.path.abspath(args.config))
    os.makedirs(config['output'], exist_ok=True)
    with open(os.path.join(config['output'], "opt_config.json"), 'w') as f:
        json.dump(config, f, indent=4)
    if args.forward_mode:
        if not args.patterns:
            raise ValueError("In forward mode, you must specify the patterns file.")
        patterns = np.load(args.patterns)['patterns']
        optimize(config, patterns_fwd=patterns)
    else:
        optimize(config)


if __name__ == "__main__":
    main()
