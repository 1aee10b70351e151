"""ctypes binding of libtvam.so (include/tvam.h).

The GPU path has no fallback: if the HIP library is missing or fails to load,
every call raises.  ``TvamDesc`` mirrors ``struct tvam_desc`` field for field.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TVAM_LIB") or os.path.join(_HERE, "libtvam.so")  # TVAM_LIB: a variant build

ABI_VERSION = 12

TVAM_OK = 0
TVAM_ERR_INVALID = -1
TVAM_ERR_UNSUPPORTED = -2
TVAM_ERR_HIP = -3
TVAM_ERR_TOO_LARGE = -4

PROJECTOR_COLLIMATED = 0
VIAL_INDEX_MATCHED = 0
VIAL_CYLINDRICAL = 1
VIAL_SQUARE = 2
PHASE_ISOTROPIC = 0
PHASE_RAYLEIGH = 1
PHASE_HG = 2
SENSOR_DDA = 0
SENSOR_RATIO = 1
SENSOR_DELTA = 2

FLAG_NO_ZERO_SKIP = 1
FLAG_FWD_STATS = 2
FLAG_NO_PLANAR = 4
FLAG_RAY_FWD = 8
FLAG_SCATTER_ATOMIC = 16
LBFGS_WORK_DOUBLES = 2048 * 64


class TvamDesc(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("projector_type", ctypes.c_int32),
        ("n_patterns", ctypes.c_int32),
        ("res_x", ctypes.c_int32),
        ("res_y", ctypes.c_int32),
        ("crop_x", ctypes.c_int32),
        ("crop_y", ctypes.c_int32),
        ("crop_offset_x", ctypes.c_int32),
        ("crop_offset_y", ctypes.c_int32),
        ("pixel_size_x", ctypes.c_float),
        ("pixel_size_y", ctypes.c_float),
        ("distance", ctypes.c_float),
        ("clockwise", ctypes.c_int32),
        ("sensor_type", ctypes.c_int32),
        ("bbox_min", ctypes.c_float * 3),
        ("bbox_max", ctypes.c_float * 3),
        ("film_res", ctypes.c_int32 * 3),
        ("film_channels", ctypes.c_int32),
        ("vial_type", ctypes.c_int32),
        ("vial_r", ctypes.c_float),
        ("vial_r_ext", ctypes.c_float),
        ("vial_height", ctypes.c_float),
        ("vial_ior", ctypes.c_float),
        ("medium_ior", ctypes.c_float),
        ("sigma_t", ctypes.c_float),
        ("albedo", ctypes.c_float),
        ("print_time", ctypes.c_float),
        ("regular_sampling", ctypes.c_int32),
        ("sample_time", ctypes.c_int32),
        ("max_depth", ctypes.c_int32),
        ("rr_depth", ctypes.c_int32),
        ("transmission_only", ctypes.c_int32),
        ("angle_begin", ctypes.c_int32),
        ("angle_end", ctypes.c_int32),
        ("tile", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("slab_begin", ctypes.c_int32),
        ("slab_end", ctypes.c_int32),
        ("phase_type", ctypes.c_int32),
        ("phase_g", ctypes.c_float),
        ("occluder_tris", ctypes.c_void_p),
        ("n_occluder_tris", ctypes.c_int32),
        ("target_tris", ctypes.c_void_p),
        ("n_target_tris", ctypes.c_int32),
        ("majorant", ctypes.c_float),
        ("reserved0", ctypes.c_int32),
        ("active_base", ctypes.c_int64),
        ("active_total", ctypes.c_int64),
    ]

    def copy(self) -> "TvamDesc":
        d = TvamDesc()
        ctypes.pointer(d)[0] = self
        for keep in ("_occluders", "_targets"):  # keep the triangle arrays alive with the copy
            if hasattr(self, keep):
                setattr(d, keep, getattr(self, keep))
        return d

    def set_target(self, tris) -> None:
        """Target mesh triangles [n][3][3] (float32, host, world space) for surface-aware films."""
        import numpy as np
        t = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 3, 3)
        self._targets = t
        self.target_tris = t.ctypes.data if t.size else None
        self.n_target_tris = int(t.shape[0])

    def set_occluders(self, tris) -> None:
        """Occluder triangles [n][3][3] (float32, host); the desc keeps the array alive."""
        import numpy as np
        t = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 3, 3)
        self._occluders = t
        self.occluder_tris = t.ctypes.data if t.size else None
        self.n_occluder_tris = int(t.shape[0])

    def as_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = list(v) if isinstance(v, ctypes.Array) else v
        return out


# Entry points declared in include/tvam.h, with their ctypes signatures.
_P = ctypes.c_void_p
EXPORTS = {
    "tvam_desc_init": (None, [ctypes.POINTER(TvamDesc)]),
    "tvam_plan_create": (ctypes.c_int, [ctypes.POINTER(TvamDesc), ctypes.c_int, ctypes.POINTER(_P)]),
    "tvam_plan_destroy": (None, [_P]),
    "tvam_forward": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _P, _P]),
    "tvam_adjoint": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _P, _P]),
    "tvam_forward_slices": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "tvam_plan_fwd_chunk": (ctypes.c_int, [_P]),
    "tvam_lbfgs_history": (ctypes.c_int, [ctypes.c_uint64, _P, _P, _P, _P, ctypes.c_int32, _P, _P, _P, _P, _P, _P,
                                          _P]),
    "tvam_lbfgs_direction": (ctypes.c_int, [ctypes.c_uint64, _P, ctypes.c_int32, _P, _P, ctypes.c_float, _P, _P, _P,
                                            _P]),
    "tvam_lbfgs_coef": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, _P, _P]),
    "tvam_lbfgs_direction_dev": (ctypes.c_int, [ctypes.c_uint64, _P, ctypes.c_int32, _P, _P, _P, _P, _P]),
    "tvam_lbfgs_history_rows": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _P,
                                               _P, _P, _P, ctypes.c_int32, _P, _P, _P, _P, _P, _P, _P]),
    "tvam_lbfgs_direction_rows": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _P,
                                                 ctypes.c_int32, _P, _P, _P, _P, _P]),
    "tvam_axpy_clamp": (ctypes.c_int, [ctypes.c_uint64, _P, ctypes.c_float, _P, ctypes.c_float, _P, _P]),
    "tvam_axpy_clamp_dev": (ctypes.c_int, [ctypes.c_uint64, _P, _P, _P, ctypes.c_float, _P, _P, _P]),
    "tvam_lbfgs_armijo": (ctypes.c_int, [ctypes.c_int32, ctypes.c_double, _P, _P, ctypes.c_double, ctypes.c_double,
                                         _P, ctypes.c_double, _P, _P, _P]),
    "tvam_row_slices": (ctypes.c_int, [ctypes.POINTER(TvamDesc), _P]),
    "tvam_plan_path": (ctypes.c_int, [_P]),
    "tvam_adjoint_slices": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, _P, _P]),
    "tvam_plan_adj_chunk": (ctypes.c_int, [_P]),
    "tvam_plan_set_active": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int64]),
    "tvam_compute_volume": (ctypes.c_int, [_P, ctypes.c_uint32, _P, _P]),
    "tvam_plan_set_volumes": (ctypes.c_int, [_P, _P]),
    "tvam_radon": (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, _P, _P]),
    "tvam_count_visits": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]),
    "tvam_plan_stats": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "tvam_discretize": (ctypes.c_int, [ctypes.POINTER(TvamDesc), _P, _P]),
    "tvam_plan_fwd_scale": (ctypes.c_int, [_P, _P]),
    "tvam_plan_bin_stats": (ctypes.c_int, [_P, _P]),
    "tvam_plan_tile_stats": (ctypes.c_int, [_P, _P]),
    "tvam_plan_kernel_time": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_int64)]),
    "tvam_loss_threshold": (
        ctypes.c_int,
        [_P, _P, ctypes.c_float, _P, ctypes.c_uint64, ctypes.c_int32, ctypes.c_float, ctypes.c_float,
         ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P, _P],
    ),
    "tvam_loss_threshold_probes": (
        ctypes.c_int,
        [_P, _P, _P, ctypes.c_int32, _P, ctypes.c_uint64, ctypes.c_int32, ctypes.c_float, ctypes.c_float,
         ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P],
    ),
    "tvam_target_mask": (ctypes.c_int, [_P, ctypes.c_uint64, _P, _P]),
    "tvam_loss_threshold_mask": (
        ctypes.c_int,
        [_P, _P, ctypes.c_float, _P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_float, ctypes.c_float,
         ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P, _P],
    ),
    "tvam_loss_threshold_probes_mask": (
        ctypes.c_int,
        [_P, _P, _P, ctypes.c_int32, _P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_float,
         ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P],
    ),
    "tvam_last_error": (ctypes.c_char_p, []),
    "tvam_abi_version": (ctypes.c_int, []),
}

_lib = None
_lock = threading.Lock()


class TvamError(RuntimeError):
    pass


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libtvam.so (no fallback: raises if it is absent)."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise TvamError(
                f"libtvam.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or drtvam_amd/csrc/build.sh (there is no CPU fallback)"
            )
        lib = ctypes.CDLL(p)
        # the version first: a library built before an export was added fails with this message,
        # not an AttributeError from the binding loop
        ver = getattr(lib, "tvam_abi_version", None)
        if ver is None:
            raise TvamError(f"{p} exports no tvam_abi_version; rebuild it")
        ver.restype, ver.argtypes = ctypes.c_int, []
        if ver() != ABI_VERSION:
            raise TvamError(f"libtvam.so ABI version mismatch ({ver()} != {ABI_VERSION}); rebuild it")
        for name, (res, args) in EXPORTS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                raise TvamError(f"libtvam.so lacks {name} (ABI {ABI_VERSION}); rebuild it")
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def check(rc: int) -> None:
    if rc == TVAM_OK:
        return
    msg = load_library().tvam_last_error().decode(errors="replace")
    if rc in (TVAM_ERR_INVALID, TVAM_ERR_UNSUPPORTED):
        raise ValueError(msg)
    if rc == TVAM_ERR_TOO_LARGE:
        raise Exception(msg)
    raise TvamError(msg)


def default_desc() -> TvamDesc:
    d = TvamDesc()
    load_library().tvam_desc_init(ctypes.byref(d))
    return d
