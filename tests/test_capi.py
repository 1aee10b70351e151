"""C-ABI boundary checks that need no GPU: libtvam.so loads, exports every
entry point include/tvam.h declares, and validates descriptors with the
reference's error semantics before touching the HIP runtime."""
import ctypes
import os
import re

import pytest

from drtvam_amd import _abi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "tvam.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tvam_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _abi.load_library()
    names = declared_functions()
    assert "tvam_forward" in names and "tvam_adjoint" in names and len(names) >= 9
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_abi.EXPORTS), "ctypes signature table out of sync with include/tvam.h"


def test_desc_layout_matches_header(tmp_path):
    """The ctypes mirror has the C struct's size and field offsets (compiled with gcc)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    names = [n for n, _ in _abi.TvamDesc._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "tvam.h"\nint main(void){\n'
                   'printf("%zu\\n", sizeof(tvam_desc));\n' +
                   "".join(f'printf("%zu\\n", offsetof(tvam_desc, {n}));\n' for n in names) + "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert ctypes.sizeof(_abi.TvamDesc) == vals[0]
    for n, off in zip(names, vals[1:]):
        assert getattr(_abi.TvamDesc, n).offset == off, n


def test_desc_defaults_follow_reference():
    d = _abi.default_desc()
    assert d.abi_version == _abi.ABI_VERSION
    assert d.n_patterns == 1000 and d.res_x == 256 and d.res_y == 256  # projector.py:73-75
    assert list(d.film_res) == [256, 256, 256]                          # film.py:9-11
    assert d.print_time == 1.0 and d.transmission_only == 1            # common.py:13,19
    assert d.max_depth == 6 and d.rr_depth == 6                          # optimize.py:99-100
    assert d.vial_height == 40.0                                         # geometry.py:80


@pytest.mark.parametrize("field,value,msg", [
    ("vial_r", 0.0, "radius"),
    ("crop_x", 300, "Crop resolution"),
    ("crop_offset_x", 100, "crop offset"),
    ("film_channels", 2, "No target shape"),  # surface-aware film without a target mesh (sensor.py:60-61)
    ("film_channels", 3, "film_channels"),
    ("albedo", 0.5, "scattering"),
    ("abi_version", 99, "abi_version"),
])
def test_plan_create_rejects_invalid_desc(field, value, msg):
    lib = _abi.load_library()
    d = _abi.default_desc()
    d.vial_r = 8.0
    setattr(d, field, value)
    plan = ctypes.c_void_p()
    rc = lib.tvam_plan_create(ctypes.byref(d), 0, ctypes.byref(plan))
    assert rc in (_abi.TVAM_ERR_INVALID, _abi.TVAM_ERR_UNSUPPORTED)
    assert not plan.value
    assert msg in lib.tvam_last_error().decode()
    with pytest.raises(ValueError, match=msg):
        _abi.check(rc)


def test_round4_vector_entry_points_validate_before_hip():
    """tvam_lbfgs_coef / _direction_rows / _history_rows and tvam_adjoint_slices reject bad
    arguments with TVAM_ERR_INVALID (or UNSUPPORTED) before any HIP call, with a message."""
    lib = _abi.load_library()
    buf = (ctypes.c_double * 256)()
    f32 = (ctypes.c_float * 64)()
    order = (ctypes.c_int32 * 8)(0, 1, 2, 3, 4, 5, 6, 7)
    bad_order = (ctypes.c_int32 * 8)(0, 9, 0, 0, 0, 0, 0, 0)
    ptrs = (ctypes.c_void_p * 8)(*([ctypes.addressof(f32)] * 8))
    p = ctypes.addressof(buf)
    q = ctypes.addressof(f32)
    cases = [
        lib.tvam_lbfgs_coef(9, 0, 0, order, p, p, q, p, None),             # h > 8
        lib.tvam_lbfgs_coef(2, 0, 0, bad_order, p, p, q, p, None),         # slot out of the ring
        lib.tvam_lbfgs_coef(0, 1, 0, order, p, p, q, p, None),             # a new pair needs h >= 1
        lib.tvam_lbfgs_coef(2, 0, 0, order, None, p, q, p, None),          # null dots
        lib.tvam_lbfgs_direction_rows(0, 4, 8, 0, q, 1, ptrs, ptrs, q, q, None),     # no segments
        lib.tvam_lbfgs_direction_rows(2, 6, 8, 0, q, 1, ptrs, ptrs, q, q, None),     # length not a multiple of 4
        lib.tvam_lbfgs_direction_rows(2, 12, 8, 0, q, 1, ptrs, ptrs, q, q, None),    # segment longer than stride
        lib.tvam_lbfgs_history_rows(2, 4, 8, 2, q, q, q, q, 1, ptrs, ptrs, q, q, p, p, None),  # offset misaligned
        lib.tvam_lbfgs_history_rows(1, 4, 8, 0, q, q, q, q, 8, ptrs, ptrs, q, q, p, p, None),  # h > 7
        lib.tvam_adjoint_slices(None, q, 16, 0, 8, 0, 4, q, None),                    # null plan
    ]
    for i, rc in enumerate(cases):
        assert rc in (_abi.TVAM_ERR_INVALID, _abi.TVAM_ERR_UNSUPPORTED), (i, rc)
    assert lib.tvam_last_error()
