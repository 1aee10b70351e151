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


def test_desc_layout_matches_header():
    # the ctypes mirror must have the same size as the C struct: count fields in the header
    src = open(HEADER).read()
    body = src[src.index("typedef struct tvam_desc {"):src.index("} tvam_desc;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    n = 0
    for line in body.splitlines():
        m = re.match(r"\s*(int32_t|float)\s+(.*);", line)
        if not m:
            continue
        for decl in m.group(2).split(","):
            arr = re.search(r"\[(\d+)\]", decl)
            n += int(arr.group(1)) if arr else 1
    assert ctypes.sizeof(_abi.TvamDesc) == 4 * n


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
    ("film_channels", 2, "surface-aware"),
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
