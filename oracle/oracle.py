"""ctypes wrapper of the CPU oracle (oracle/tvam_oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg (as the timed CPU port).  The product
package drtvam_amd never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
import threading
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "liboracle.so")

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(_HERE, "tvam_oracle.c")):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        from drtvam_amd._abi import TvamDesc  # the descriptor struct is the shared ABI

        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        D = ctypes.POINTER(TvamDesc)
        L.oracle_forward.restype = ctypes.c_int
        L.oracle_forward.argtypes = [D, P, P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, P, P, ctypes.c_int]
        L.oracle_adjoint.restype = ctypes.c_int
        L.oracle_adjoint.argtypes = [D, P, P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, P, P, ctypes.c_int]
        L.oracle_ray.restype = ctypes.c_int
        L.oracle_ray.argtypes = [D, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, P]
        L.oracle_forward_part.restype = ctypes.c_int
        L.oracle_forward_part.argtypes = L.oracle_forward.argtypes + [ctypes.c_int]
        L.oracle_phase.restype = ctypes.c_int
        L.oracle_phase.argtypes = [D, P, ctypes.c_float, ctypes.c_float, P]
        L.oracle_radon.restype = ctypes.c_int
        L.oracle_radon.argtypes = [D, P, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P, ctypes.c_int]
        L.oracle_forward_surface.restype = ctypes.c_int
        L.oracle_forward_surface.argtypes = [D, P, P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, P, P, P,
                                             ctypes.c_int]
        L.oracle_adjoint_surface.restype = ctypes.c_int
        L.oracle_adjoint_surface.argtypes = L.oracle_forward_surface.argtypes
        L.oracle_compute_volume.restype = ctypes.c_int
        L.oracle_compute_volume.argtypes = [D, ctypes.c_uint32, P, ctypes.c_int]
        L.oracle_frozen_axes.restype = ctypes.c_uint64
        L.oracle_frozen_axes.argtypes = [ctypes.c_int]
        L.oracle_discretize.restype = ctypes.c_int
        L.oracle_discretize.argtypes = [D, P, ctypes.c_int]
        L.oracle_forward_streams.restype = ctypes.c_int
        L.oracle_forward_streams.argtypes = [D, P, P, P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, P, P,
                                             ctypes.c_int]
        L.oracle_adjoint_streams.restype = ctypes.c_int
        L.oracle_adjoint_streams.argtypes = L.oracle_forward_streams.argtypes
        L.oracle_dda_ray.restype = ctypes.c_int
        L.oracle_dda_ray.argtypes = [D, P, P, ctypes.c_float, ctypes.c_double, P, P]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _call(name, fn, *args):
    """fn(*args) (a ctypes call: it releases the GIL) on a worker thread; while it runs longer than
    50 s, one progress line per 50 s on the process's real stderr (a full-size scattering oracle
    pass takes minutes of silent CPU work, which a hang watchdog would otherwise take for a hang)."""
    out = {}
    th = threading.Thread(target=lambda: out.__setitem__("rc", fn(*args)), daemon=True)
    t0 = time.perf_counter()
    th.start()
    while True:
        th.join(50.0)
        if not th.is_alive():
            break
        print(f"[oracle] {name}: running for {time.perf_counter() - t0:.0f} s", file=sys.__stderr__, flush=True)
    return out["rc"]


def film_shape(desc):
    rx, ry, rz = desc.film_res
    return (rz, ry, rx)


def forward(desc, active_data, active_pixels=None, spp=1, seed=0, nthreads=1, part=-1, streams=None):
    """Dose [z, y, x] (float64) and the DDA visit count of one forward pass.
    Scattering media: part=1 keeps only each path's first medium segment, part=0 the rest.
    streams: per active entry, its position in a larger set (sampler streams streams[i] * spp + k):
    a subset of a plan's dense shard traced with the shard's own streams."""
    data = np.ascontiguousarray(active_data, dtype=np.float32)
    pix = None if active_pixels is None else np.ascontiguousarray(active_pixels, dtype=np.uint32)
    dose = np.zeros(film_shape(desc), dtype=np.float64)
    visits = ctypes.c_uint64(0)
    if streams is not None:
        st = np.ascontiguousarray(streams, dtype=np.uint64)
        assert pix is not None and st.size == data.size == pix.size and part == -1
        rc = _call("forward", lib().oracle_forward_streams, ctypes.byref(desc), _ptr(data), _ptr(pix), _ptr(st), data.size, spp, seed,
                                          _ptr(dose), ctypes.cast(ctypes.byref(visits), ctypes.c_void_p), nthreads)
        if rc:
            raise ValueError(f"oracle_forward_streams failed ({rc})")
        return dose, visits.value
    rc = _call("forward", lib().oracle_forward_part, ctypes.byref(desc), _ptr(data), _ptr(pix), data.size, spp, seed, _ptr(dose),
                                   ctypes.cast(ctypes.byref(visits), ctypes.c_void_p), nthreads, part)
    if rc:
        raise ValueError(f"oracle_forward failed ({rc})")
    return dose, visits.value


def adjoint(desc, grad_dose, active_pixels=None, n_active=None, spp=1, seed=0, nthreads=1, streams=None):
    """Gradient w.r.t. active_data (float64) of <grad_dose, forward(.)>.  streams: as in forward()."""
    g = np.ascontiguousarray(grad_dose, dtype=np.float32).reshape(film_shape(desc))
    pix = None if active_pixels is None else np.ascontiguousarray(active_pixels, dtype=np.uint32)
    if n_active is None:
        n_active = pix.size if pix is not None else desc.n_patterns * desc.crop_y * desc.crop_x
    out = np.zeros(n_active, dtype=np.float64)
    visits = ctypes.c_uint64(0)
    if streams is not None:
        st = np.ascontiguousarray(streams, dtype=np.uint64)
        assert pix is not None and st.size == pix.size == n_active
        rc = _call("adjoint", lib().oracle_adjoint_streams, ctypes.byref(desc), _ptr(g), _ptr(pix), _ptr(st), n_active, spp, seed,
                                          _ptr(out), ctypes.cast(ctypes.byref(visits), ctypes.c_void_p), nthreads)
        if rc:
            raise ValueError(f"oracle_adjoint_streams failed ({rc})")
        return out, visits.value
    rc = _call("adjoint", lib().oracle_adjoint, ctypes.byref(desc), _ptr(g), _ptr(pix), n_active, spp, seed, _ptr(out),
                              ctypes.cast(ctypes.byref(visits), ctypes.c_void_p), nthreads)
    if rc:
        raise ValueError(f"oracle_adjoint failed ({rc})")
    return out, visits.value


def ray(desc, pixel, wave_index=0, seed=0):
    """Projector ray of one sample and its medium segment (o2, d2, maxt) + interface weight."""
    out = np.zeros(15, dtype=np.float32)
    lib().oracle_ray(ctypes.byref(desc), pixel, wave_index, seed, _ptr(out))
    return {"o": out[0:3].copy(), "d": out[3:6].copy(), "hit": bool(out[6]), "o2": out[7:10].copy(),
            "maxt": float(out[10]), "d2": out[11:14].copy(), "weight": float(out[14])}


def radon(desc, target_tris, spp=4, seed=0, max_depth=5, nthreads=1):
    """Radon filter image (float64, dense crop order) for world-space target triangles [n, 3, 3]."""
    tris = np.ascontiguousarray(target_tris, dtype=np.float32).reshape(-1, 9)
    out = np.zeros(desc.n_patterns * desc.crop_y * desc.crop_x, dtype=np.float64)
    rc = lib().oracle_radon(ctypes.byref(desc), _ptr(tris), tris.shape[0], spp, seed, max_depth, _ptr(out), nthreads)
    if rc:
        raise ValueError(f"oracle_radon failed ({rc})")
    return out


def phase(desc, d, u1, u2):
    """Scattered direction for a ray of direction d (the desc's phase function)."""
    d = np.ascontiguousarray(d, dtype=np.float32)
    wo = np.zeros(3, dtype=np.float32)
    lib().oracle_phase(ctypes.byref(desc), _ptr(d), u1, u2, _ptr(wo))
    return wo


def dda_ray(desc, o, d, maxt, em=1.0):
    o = np.ascontiguousarray(o, dtype=np.float32)
    d = np.ascontiguousarray(d, dtype=np.float32)
    film = np.zeros(film_shape(desc), dtype=np.float64)
    visits = ctypes.c_uint64(0)
    lib().oracle_dda_ray(ctypes.byref(desc), _ptr(o), _ptr(d), maxt, em, _ptr(film),
                         ctypes.cast(ctypes.byref(visits), ctypes.c_void_p))
    return film, visits.value


def inv_volumes(volumes):
    """1 / volume per (voxel, channel), 0 where the volume is 0 (volume.py:41-42), fp32."""
    v = np.asarray(volumes, dtype=np.float32)
    out = np.zeros_like(v)
    nz = v != 0
    out[nz] = np.float32(1.0) / v[nz]
    return out


def compute_volume(desc, sample_count=2 ** 14, nthreads=1):
    """Surface-aware voxel volumes [z, y, x, 2] (inside, outside) of the desc's target mesh."""
    out = np.zeros(film_shape(desc) + (2,), dtype=np.float32)
    rc = lib().oracle_compute_volume(ctypes.byref(desc), sample_count, _ptr(out), nthreads)
    if rc:
        raise ValueError(f"oracle_compute_volume failed ({rc})")
    return out


def frozen_axes(reset=True):
    """Number of DDA segments (since the last reset) that started with a valid axis whose first
    crossing time rounded negative, so that axis never steps (sensor.py:358)."""
    return int(lib().oracle_frozen_axes(1 if reset else 0))


def discretize(desc, nthreads=1):
    """Binary target occupancy [z, y, x] (float32) of the desc's target mesh on its film grid
    (utils.py:83-128: one sampled direction per voxel centre)."""
    out = np.zeros(film_shape(desc), dtype=np.float32)
    rc = lib().oracle_discretize(ctypes.byref(desc), _ptr(out), nthreads)
    if rc:
        raise ValueError(f"oracle_discretize failed ({rc})")
    return out


def forward_surface(desc, active_data, volumes, active_pixels=None, spp=1, seed=0, nthreads=1):
    """Surface-aware dose [z, y, x, 2] (float64) = film / volumes per channel, and the visit count."""
    data = np.ascontiguousarray(active_data, dtype=np.float32)
    pix = None if active_pixels is None else np.ascontiguousarray(active_pixels, dtype=np.uint32)
    iv = np.ascontiguousarray(inv_volumes(volumes))
    dose = np.zeros(film_shape(desc) + (2,), dtype=np.float64)
    visits = ctypes.c_uint64(0)
    rc = lib().oracle_forward_surface(ctypes.byref(desc), _ptr(data), _ptr(pix), data.size, spp, seed, _ptr(iv),
                                      _ptr(dose), ctypes.cast(ctypes.byref(visits), ctypes.c_void_p), nthreads)
    if rc:
        raise ValueError(f"oracle_forward_surface failed ({rc})")
    return dose, visits.value


def adjoint_surface(desc, grad_dose, volumes, active_pixels=None, n_active=None, spp=1, seed=0, nthreads=1):
    """Gradient w.r.t. active_data (float64) of <grad_dose, forward_surface(.)>."""
    g = np.ascontiguousarray(grad_dose, dtype=np.float32).reshape(film_shape(desc) + (2,))
    pix = None if active_pixels is None else np.ascontiguousarray(active_pixels, dtype=np.uint32)
    if n_active is None:
        n_active = pix.size if pix is not None else desc.n_patterns * desc.crop_y * desc.crop_x
    iv = np.ascontiguousarray(inv_volumes(volumes))
    out = np.zeros(n_active, dtype=np.float64)
    visits = ctypes.c_uint64(0)
    rc = lib().oracle_adjoint_surface(ctypes.byref(desc), _ptr(g), _ptr(pix), n_active, spp, seed, _ptr(iv),
                                      _ptr(out), ctypes.cast(ctypes.byref(visits), ctypes.c_void_p), nthreads)
    if rc:
        raise ValueError(f"oracle_adjoint_surface failed ({rc})")
    return out, visits.value
