"""EXR image I/O (Mitsuba Bitmap's role in utils.py:29-46 and projector.py:24-37).

No OpenEXR library is installed here, so parity is unpinned against a
third-party reader: the checks are round trips through every compression the
writer/reader support, the file layout of the OpenEXR 2 spec (magic, version,
sorted channel list, offset table, chunk headers) parsed by hand, a hand-made
RLE block, and reshape_grid's mosaic order against the reference's formula.
"""
import os
import struct

import numpy as np
import pytest

from drtvam_amd import exr
from drtvam_amd.projector import load_patterns
from drtvam_amd.utils import reshape_grid, save_img, save_vol


@pytest.mark.parametrize("comp", [exr.NO_COMPRESSION, exr.ZIPS_COMPRESSION, exr.ZIP_COMPRESSION])
@pytest.mark.parametrize("shape", [(7, 5), (33, 17, 1), (20, 9, 2), (16, 16, 3), (3, 4, 4), (5, 6, 5)])
def test_round_trip(tmp_path, comp, shape):
    rng = np.random.default_rng(sum(shape) + comp)
    img = rng.standard_normal(shape).astype(np.float32)
    img.reshape(-1)[::7] = 0.0  # runs that compress
    path = str(tmp_path / "a.exr")
    exr.write_exr(path, img, compression=comp)
    back, names = exr.read_exr(path, with_names=True)
    want = img if img.ndim == 3 else img[..., None]
    assert back.dtype == np.float32 and back.shape == want.shape
    np.testing.assert_array_equal(back, want)
    assert names == exr.channel_names(want.shape[2])


def test_file_layout(tmp_path):
    """Magic, version 2 (single-part scanline), channel list sorted by name, FLOAT pixels,
    offset table pointing at (y, size) chunk headers, one scanline per chunk uncompressed."""
    img = np.arange(2 * 3 * 2, dtype=np.float32).reshape(2, 3, 2)  # channels Y, A
    path = str(tmp_path / "b.exr")
    exr.write_exr(path, img, compression=exr.NO_COMPRESSION)
    buf = open(path, "rb").read()
    assert struct.unpack_from("<ii", buf, 0) == (20000630, 2)
    i = buf.index(b"channels\0chlist\0")
    (size,) = struct.unpack_from("<i", buf, i + 16)
    chl = buf[i + 20:i + 20 + size]
    assert chl == b"A\0" + struct.pack("<iB3xii", 2, 0, 1, 1) + b"Y\0" + struct.pack("<iB3xii", 2, 0, 1, 1) + b"\0"
    hdr_end = buf.index(b"screenWindowWidth\0float\0") + len(b"screenWindowWidth\0float\0") + 8 + 1
    offs = struct.unpack_from("<2Q", buf, hdr_end)
    for y, off in enumerate(offs):
        yy, sz = struct.unpack_from("<ii", buf, off)
        assert (yy, sz) == (y, 2 * 3 * 4)
        a = np.frombuffer(buf, dtype="<f4", count=3, offset=off + 8)     # channel A of line y
        yv = np.frombuffer(buf, dtype="<f4", count=3, offset=off + 20)   # channel Y of line y
        np.testing.assert_array_equal(a, img[y, :, 1])
        np.testing.assert_array_equal(yv, img[y, :, 0])


def test_rle_block(tmp_path):
    """A hand-encoded RLE scanline (predictor + interleave + runs) decodes to its pixels."""
    vals = np.array([1.0, 1.0, 1.0, 2.5], dtype="<f4")
    raw = np.frombuffer(vals.tobytes(), dtype=np.uint8)
    t = np.concatenate([raw[0::2], raw[1::2]]).astype(np.int16)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128 + 256) % 256
    enc = bytearray()
    for b in d.astype(np.uint8):  # literal runs of 1 byte each: count -1, byte
        enc += struct.pack("<b", -1) + bytes([int(b)])
    assert exr._rle_decode(bytes(enc), raw.size) == raw.tobytes()


def test_reshape_grid_order():
    """rows = ceil(sqrt(n)); slice k lands at mosaic tile (k // rows, k % rows) (utils.py:13-27)."""
    vol = np.arange(5 * 2 * 3, dtype=np.float32).reshape(5, 2, 3)
    g = reshape_grid(vol)
    assert g.shape == (3 * 2, 3 * 3, 1)
    for k in range(9):
        r, c = divmod(k, 3)
        want = vol[k] if k < 5 else np.zeros((2, 3))
        np.testing.assert_array_equal(g[r * 2:(r + 1) * 2, c * 3:(c + 1) * 3, 0], want)


def test_save_vol_and_pattern_dir(tmp_path):
    vol = np.random.default_rng(0).uniform(size=(4, 3, 5, 1)).astype(np.float32)
    save_vol(vol, str(tmp_path / "final.exr"))
    np.testing.assert_array_equal(exr.read_exr(str(tmp_path / "final.exr")), reshape_grid(vol).astype(np.float32))
    d = tmp_path / "patterns"
    os.makedirs(d)
    pats = np.random.default_rng(1).uniform(size=(3, 6, 7)).astype(np.float32)
    for i in range(3):
        save_img(pats[i], str(d / f"{i:04d}.exr"))
    np.testing.assert_array_equal(load_patterns(str(d)), pats)
    save_img(np.zeros((5, 7), np.float32), str(d / "0003.exr"))
    with pytest.raises(ValueError, match="different resolution"):
        load_patterns(str(d))
    with pytest.raises(ValueError, match="No patterns found"):
        load_patterns(str(tmp_path / "empty_dir_does_not_exist"))
