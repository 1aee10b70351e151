"""Device-side projection engine: owns a tvam_plan and exposes the forward /
adjoint projections as torch operations.

``TvamRender`` plays the role of Mitsuba's ``mi.render`` custom op
(optimize.py:216, :294): its forward is VolumeIntegrator.render
(integrators/volume.py:18-56) and its backward is render_backward
(integrators/volume.py:97-134).  Both run the HIP kernels of libtvam.so; there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _abi


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def derive_seed_grad(seed: int) -> int:
    """Seed of the adjoint pass when none is given (decorrelated from the primal)."""
    v0, v1 = seed & 0xFFFFFFFF, 1
    s = 0
    for _ in range(4):
        s = (s + 0x9E3779B9) & 0xFFFFFFFF
        v0 = (v0 + ((((v1 << 4) & 0xFFFFFFFF) + 0xA341316C) ^ ((v1 + s) & 0xFFFFFFFF) ^ ((v1 >> 5) + 0xC8013EA4))) & 0xFFFFFFFF
        v1 = (v1 + ((((v0 << 4) & 0xFFFFFFFF) + 0xAD90777D) ^ ((v0 + s) & 0xFFFFFFFF) ^ ((v0 >> 5) + 0x7E95761E))) & 0xFFFFFFFF
    return v0


class Projection:
    """One tvam_plan (scene tables) bound to one GPU."""

    def __init__(self, desc: _abi.TvamDesc, device: Optional[torch.device] = None):
        if not torch.cuda.is_available():
            raise _abi.TvamError("the TVAM projection engine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _abi.load_library()
        self.desc = desc.copy()
        self.device = torch.device("cuda") if device is None else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        plan = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_plan_create(ctypes.byref(self.desc), self.device.index, ctypes.byref(plan)))
        self._plan = plan
        rx, ry, rz = self.desc.film_res
        if self.desc.slab_end >= 0:  # film slab of this plan (z-slab sharding)
            rz = self.desc.slab_end - self.desc.slab_begin
        self.film_shape = (rz, ry, rx, self.desc.film_channels)
        self.n_dense = self.desc.n_patterns * self.desc.crop_y * self.desc.crop_x

    def close(self):
        if getattr(self, "_plan", None) is not None and self._plan.value:
            self.lib.tvam_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check_tensor(self, t: torch.Tensor, dtype, name):
        if t.device != self.device or t.dtype != dtype or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {dtype} tensor on {self.device}")

    def _check_pixels(self, active_pixels: torch.Tensor):
        """The plan keeps a sparse set's ray records keyed on the active_pixels pointer and count.
        A pointer alone does not name a set: a freed tensor's address can be handed to a new one.
        So the projection holds the last tensor it was given (its storage cannot be reused while
        held) and drops the records (tvam_plan_set_active) whenever a call brings another tensor
        object, or the same tensor changed in place (new torch version)."""
        self._check_tensor(active_pixels, torch.int32, "active_pixels")
        ver = active_pixels._version
        last = getattr(self, "_pix_last", None)
        if last is not None and (last[0] is not active_pixels or last[1] != ver):
            self.set_active(self.desc.active_base, self.desc.active_total)
        self._pix_last = (active_pixels, ver)

    def forward(self, active_data: torch.Tensor, active_pixels: Optional[torch.Tensor] = None, spp: int = 1,
                seed: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        self._check_tensor(active_data, torch.float32, "active_data")
        if active_pixels is not None:
            self._check_pixels(active_pixels)
        if out is None:
            out = torch.empty(self.film_shape, dtype=torch.float32, device=self.device)
        self._check_tensor(out, torch.float32, "dose")
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_forward(
                self._plan, active_data.data_ptr(), None if active_pixels is None else active_pixels.data_ptr(),
                active_data.numel(), spp, seed & 0xFFFFFFFF, out.data_ptr(), _stream_ptr(self.device)))
        return out

    def forward_slices(self, active_data: torch.Tensor, active_pixels: Optional[torch.Tensor], spp: int, seed: int,
                       z_begin: int, z_end: int, out: torch.Tensor) -> torch.Tensor:
        """The forward of film slices [z_begin, z_end) into out (the other slices untouched)."""
        self._check_tensor(active_data, torch.float32, "active_data")
        if active_pixels is not None:
            self._check_pixels(active_pixels)
        self._check_tensor(out, torch.float32, "dose")
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_forward_slices(
                self._plan, active_data.data_ptr(), None if active_pixels is None else active_pixels.data_ptr(),
                active_data.numel(), spp, seed & 0xFFFFFFFF, int(z_begin), int(z_end), out.data_ptr(),
                _stream_ptr(self.device)))
        return out

    @property
    def fwd_chunk(self) -> int:
        """Slice granularity of forward_slices (0: not splittable)."""
        return int(self.lib.tvam_plan_fwd_chunk(self._plan))

    def adjoint(self, grad_dose: torch.Tensor, n_active: int, active_pixels: Optional[torch.Tensor] = None,
                spp: int = 1, seed: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        grad_dose = grad_dose.contiguous()
        self._check_tensor(grad_dose, torch.float32, "grad_dose")
        if grad_dose.numel() != self.film_shape[0] * self.film_shape[1] * self.film_shape[2] * self.film_shape[3]:
            raise ValueError("grad_dose has the wrong number of elements")
        if active_pixels is not None:
            self._check_pixels(active_pixels)
        if out is None:
            out = torch.empty(n_active, dtype=torch.float32, device=self.device)
        self._check_tensor(out, torch.float32, "grad_active")
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_adjoint(
                self._plan, grad_dose.data_ptr(), None if active_pixels is None else active_pixels.data_ptr(),
                n_active, spp, seed & 0xFFFFFFFF, out.data_ptr(), _stream_ptr(self.device)))
        return out

    def adjoint_slices(self, grad_dose: torch.Tensor, n_active: int, z_begin: int, z_end: int, row_begin: int,
                       row_end: int, out: torch.Tensor) -> torch.Tensor:
        """The planar adjoint of film slices [z_begin, z_end) into DMD rows [row_begin, row_end) of every
        angle of out (dense set; those rows zeroed first, the rest untouched; tvam_adjoint_slices).
        An empty row range (row_begin == row_end) zeroes nothing: the slices' contributions are added
        to out as it stands (a caller that zeroed the whole vector once)."""
        self._check_tensor(grad_dose, torch.float32, "grad_dose")
        self._check_tensor(out, torch.float32, "grad_active")
        if out.numel() != n_active:
            raise ValueError("adjoint_slices: out must hold n_active entries")
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_adjoint_slices(self._plan, grad_dose.data_ptr(), n_active, int(z_begin),
                                                    int(z_end), int(row_begin), int(row_end), out.data_ptr(),
                                                    _stream_ptr(self.device)))
        return out

    @property
    def adj_chunk(self) -> int:
        """Slice granularity of adjoint_slices (0: not available)."""
        return int(self.lib.tvam_plan_adj_chunk(self._plan))

    def set_active(self, active_base: int, active_total: int) -> None:
        """Position of this plan's first active entry in the whole active set and that set's
        size (desc.active_base / active_total): sampler streams and the ray weight of later
        calls follow the reference's whole projector.active_pixels (common.py:57-67)."""
        _abi.check(self.lib.tvam_plan_set_active(self._plan, int(active_base), int(active_total)))
        self.desc.active_base = int(active_base)
        self.desc.active_total = int(active_total)

    def compute_volume(self, sample_count: int = 2 ** 14) -> torch.Tensor:
        """Surface-aware voxel volumes [Z, Y, X, 2] (inside, outside the target mesh) of this plan's
        film (VolumetricSensor.compute_volume, sensor.py:47-110)."""
        out = torch.empty(self.film_shape[:3] + (2,), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_compute_volume(self._plan, int(sample_count), out.data_ptr(),
                                                    _stream_ptr(self.device)))
        return out

    def set_volumes(self, volumes: torch.Tensor) -> None:
        """Per-(voxel, channel) volumes of a surface-aware film (the forward divides by them,
        volume.py:41-42); the projection keeps the tensor alive."""
        self._check_tensor(volumes, torch.float32, "volumes")
        if tuple(volumes.shape) != tuple(self.film_shape):
            raise ValueError(f"volumes must have the film shape {self.film_shape}")
        _abi.check(self.lib.tvam_plan_set_volumes(self._plan, volumes.data_ptr()))
        self._volumes = volumes

    def radon(self, target_tris, spp: int = 4, seed: int = 0, max_depth: int = 5) -> torch.Tensor:
        """Radon filter image of this plan's DMD pixels (dense crop order of its shard):
        positive where a ray crosses the target inside the medium (radon.py:47-106)."""
        import numpy as np
        tris = np.ascontiguousarray(target_tris, dtype=np.float32).reshape(-1, 9)
        a0, a1 = self.desc.angle_begin, (self.desc.angle_end if self.desc.angle_end >= 0 else self.desc.n_patterns)
        out = torch.empty((a1 - a0) * self.desc.crop_y * self.desc.crop_x, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_radon(self._plan, tris.ctypes.data if tris.size else None, tris.shape[0], spp,
                                           seed & 0xFFFFFFFF, max_depth, out.data_ptr(), _stream_ptr(self.device)))
        return out

    @property
    def planar(self) -> bool:
        """True when the planar fast path (regular sampling) serves this plan's adjoint."""
        return bool(self.lib.tvam_plan_path(self._plan) & 1)

    @property
    def planar_forward(self) -> bool:
        """True when the voxel-driven planar forward serves this plan (straight rays)."""
        return bool(self.lib.tvam_plan_path(self._plan) & 2)

    def fallback_tiles(self) -> int:
        """Workgroups of the last forward that used float LDS atomics (needs FLAG_FWD_STATS)."""
        v = ctypes.c_uint64(0)
        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            _abi.check(self.lib.tvam_plan_stats(self._plan, ctypes.byref(v)))
        return int(v.value)

    def fwd_scale(self):
        """(scale, fixed) of the last ray-driven planar forward: the int32 fixed-point scale 2^e and
        whether fixed point was used (False: the overflow bound was not finite, float adds)."""
        import numpy as np
        v = np.zeros(2, dtype=np.float32)
        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            _abi.check(self.lib.tvam_plan_fwd_scale(self._plan, v.ctypes.data))
        return float(v[0]), bool(v[1] != 0.0)

    def bin_stats(self):
        """Chunking of the last brick-binned call (scattering media): a dict with the chunks of
        paths, those served from / stored into the forward bin cache, the brick entries marched,
        the paths per chunk, the device bytes of the bin cache and scratch, and the slots whose bin-fill
        walk disagreed with the record writer's closed-form brick count (0; tvam_plan_bin_stats)."""
        import numpy as np
        v = np.zeros(8, dtype=np.int64)
        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            _abi.check(self.lib.tvam_plan_bin_stats(self._plan, v.ctypes.data))
        return dict(zip(("chunks", "cached", "stored", "entries", "chunk_paths", "cache_bytes", "scratch_bytes",
                         "count_mismatch"), (int(x) for x in v)))

    def tile_stats(self):
        """Row walks of the per-ray tile kernels for the most recent ray records (jittered plans):
        the rays listed as strays (-1: no stray lists), the list capacity, the (tile, slice)
        workgroups' stray walk and main-row slot walk summed over a launch, the frozen-axis rays,
        spp, tiles and slots (tvam_plan_tile_stats)."""
        import numpy as np
        v = np.zeros(8, dtype=np.int64)
        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            _abi.check(self.lib.tvam_plan_tile_stats(self._plan, v.ctypes.data))
        return dict(zip(("strays", "stray_cap", "stray_walk", "main_walk", "frozen", "spp", "tiles", "slots"),
                        (int(x) for x in v)))

    def kernel_time(self, enable: bool):
        """Launch time of the dominant forward kernel from HIP events on its stream
        (tvam_plan_kernel_time): (total ms, launches) recorded since the previous call; enable
        starts a new measurement."""
        t = ctypes.c_double(0.0)
        n = ctypes.c_int64(0)
        with torch.cuda.device(self.device):
            _abi.check(self.lib.tvam_plan_kernel_time(self._plan, 1 if enable else 0, ctypes.byref(t), ctypes.byref(n)))
        return float(t.value), int(n.value)

    def count_visits(self, spp: int = 1, seed: int = 0) -> int:
        v = ctypes.c_uint64(0)
        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            _abi.check(self.lib.tvam_count_visits(self._plan, spp, seed & 0xFFFFFFFF, ctypes.byref(v)))
        return int(v.value)


class TvamRender(torch.autograd.Function):
    """dose = render(active_data); d loss / d active_data via the adjoint kernel."""

    @staticmethod
    def forward(ctx, active_data, proj: Projection, active_pixels, spp: int, spp_grad: int, seed: int,
                seed_grad: int):
        ctx.proj = proj
        ctx.active_pixels = active_pixels
        ctx.spp_grad = spp_grad
        ctx.seed_grad = seed_grad
        ctx.n_active = active_data.numel()
        return proj.forward(active_data.detach().contiguous(), active_pixels, spp, seed)

    @staticmethod
    def backward(ctx, grad_dose):
        g = ctx.proj.adjoint(grad_dose.contiguous(), ctx.n_active, ctx.active_pixels, ctx.spp_grad, ctx.seed_grad)
        return g, None, None, None, None, None, None


def render(proj: Projection, active_data: torch.Tensor, active_pixels: Optional[torch.Tensor] = None,
           spp: int = 1, spp_grad: Optional[int] = None, seed: int = 0, seed_grad: Optional[int] = None):
    spp_grad = spp if spp_grad is None else spp_grad
    seed_grad = derive_seed_grad(seed) if seed_grad is None else seed_grad
    return TvamRender.apply(active_data, proj, active_pixels, spp, spp_grad, seed, seed_grad)


def target_mask(target: torch.Tensor) -> torch.Tensor:
    """Bit mask of a contiguous f32 target (tvam_target_mask): int32 words, bit j of word w =
    target[32 w + j] > 0, the loss kernels' object test from 1/32 of the bytes."""
    if target.dtype != torch.float32 or not target.is_contiguous() or not target.is_cuda:
        raise ValueError("target_mask: a contiguous float32 CUDA tensor")
    n = target.numel()
    mask = torch.empty((n + 31) // 32, dtype=torch.int32, device=target.device)
    with torch.cuda.device(target.device):
        _abi.check(_abi.load_library().tvam_target_mask(target.data_ptr(), n, mask.data_ptr(),
                                                        _stream_ptr(target.device)))
    return mask


def _check_mask(mask, mask_bit0, n, dev):
    if mask.dtype != torch.int32 or not mask.is_contiguous() or mask.device != dev:
        raise ValueError(f"mask must be a contiguous int32 tensor on {dev}")
    if mask_bit0 < 0 or mask_bit0 + n > 32 * mask.numel():
        raise ValueError("mask: bits [mask_bit0, mask_bit0 + n) out of range")


def loss_threshold_probes(dose: torch.Tensor, ddose: torch.Tensor, alphas, target: torch.Tensor, K: int, tl: float,
                          tu: float, w_object: float, w_void: float, w_limit: float, scale: float,
                          mask: Optional[torch.Tensor] = None, mask_bit0: int = 0) -> torch.Tensor:
    """Fused ThresholdedLoss of dose + a * ddose for each a in alphas (<= 8): f64 device vector, one pass.
    ``mask``: target_mask() of a tensor whose elements [mask_bit0, mask_bit0 + n) are this target
    (the object test read from it instead of the f32 target)."""
    lib = _abi.load_library()
    na = len(alphas)
    if not 1 <= na <= 8:
        raise ValueError("loss_threshold_probes: 1 to 8 step sizes")
    for name, t in (("dose", dose), ("ddose", ddose), ("target", target)):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dose.device:
            raise ValueError(f"{name} must be a contiguous float32 tensor on {dose.device}")
    n = dose.numel()
    if target.numel() != n or ddose.numel() != n:
        raise ValueError("loss_threshold_probes: size mismatch")
    out = torch.zeros(na, dtype=torch.float64, device=dose.device)
    a = (ctypes.c_float * na)(*[float(v) for v in alphas])
    with torch.cuda.device(dose.device):
        if mask is not None:
            _check_mask(mask, mask_bit0, n, dose.device)
            _abi.check(lib.tvam_loss_threshold_probes_mask(
                dose.data_ptr(), ddose.data_ptr(), a, na, mask.data_ptr(), int(mask_bit0), n, int(K), float(tl),
                float(tu), float(w_object), float(w_void), float(w_limit), float(scale), out.data_ptr(),
                _stream_ptr(dose.device)))
        else:
            _abi.check(lib.tvam_loss_threshold_probes(
                dose.data_ptr(), ddose.data_ptr(), a, na, target.data_ptr(), n, int(K), float(tl), float(tu),
                float(w_object), float(w_void), float(w_limit), float(scale), out.data_ptr(), _stream_ptr(dose.device)))
    return out


def loss_threshold(dose: torch.Tensor, target: torch.Tensor, K: int, tl: float, tu: float, w_object: float,
                   w_void: float, w_limit: float, scale: float, ddose: Optional[torch.Tensor] = None,
                   alpha: float = 0.0, grad: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
                   mask_bit0: int = 0) -> torch.Tensor:
    """Fused ThresholdedLoss value (f64 device scalar) and optional dL/dx (HIP kernel); ``mask`` as in
    loss_threshold_probes."""
    lib = _abi.load_library()
    out = torch.zeros(1, dtype=torch.float64, device=dose.device)
    for name, t in (("dose", dose), ("target", target), ("ddose", ddose), ("grad", grad)):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.device != dose.device):
            raise ValueError(f"{name} must be a contiguous float32 tensor on {dose.device}")
    n = dose.numel()
    if target.numel() != n or (ddose is not None and ddose.numel() != n) or (grad is not None and grad.numel() != n):
        raise ValueError("loss_threshold: size mismatch")
    with torch.cuda.device(dose.device):
        if mask is not None:
            _check_mask(mask, mask_bit0, n, dose.device)
            _abi.check(lib.tvam_loss_threshold_mask(
                dose.data_ptr(), None if ddose is None else ddose.data_ptr(), float(alpha), mask.data_ptr(),
                int(mask_bit0), n, int(K), float(tl), float(tu), float(w_object), float(w_void), float(w_limit),
                float(scale), out.data_ptr(), None if grad is None else grad.data_ptr(), _stream_ptr(dose.device)))
        else:
            _abi.check(lib.tvam_loss_threshold(
                dose.data_ptr(), None if ddose is None else ddose.data_ptr(), float(alpha), target.data_ptr(), n,
                int(K), float(tl), float(tu), float(w_object), float(w_void), float(w_limit), float(scale),
                out.data_ptr(), None if grad is None else grad.data_ptr(), _stream_ptr(dose.device)))
    return out[0]
