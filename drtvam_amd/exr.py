"""OpenEXR scanline images: the image I/O Dr.TVAM does through Mitsuba's Bitmap.

The reference writes volumes and patterns with ``mi.Bitmap(...).write(path)``
(utils.py:29-46: ``save_img`` / ``save_vol``) and reads pattern directories
with ``mi.TensorXf(mi.Bitmap(fn))`` (projector.py:24-37).  Mitsuba is not
available here, so this module implements the part of the OpenEXR 2 file
format those calls use: single-part scanline files with FLOAT / HALF / UINT
channels, written uncompressed or ZIP-compressed, read uncompressed, RLE,
ZIPS or ZIP.  Channel naming follows Bitmap's pixel formats: 1 channel = "Y",
2 = "Y", "A", 3 = "R", "G", "B", 4 = "R", "G", "B", "A" (else "0", "1", ...).
Arrays are [height, width] or [height, width, channels], float32.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

MAGIC = 20000630
NO_COMPRESSION, RLE_COMPRESSION, ZIPS_COMPRESSION, ZIP_COMPRESSION = 0, 1, 2, 3
_LINES = {NO_COMPRESSION: 1, RLE_COMPRESSION: 1, ZIPS_COMPRESSION: 1, ZIP_COMPRESSION: 16}
_PT_UINT, _PT_HALF, _PT_FLOAT = 0, 1, 2
_PT_DTYPE = {_PT_UINT: np.dtype('<u4'), _PT_HALF: np.dtype('<f2'), _PT_FLOAT: np.dtype('<f4')}


def channel_names(c: int):
    """Mitsuba Bitmap channel names of a c-channel tensor (Y, YA, RGB, RGBA, multichannel)."""
    return {1: ["Y"], 2: ["Y", "A"], 3: ["R", "G", "B"], 4: ["R", "G", "B", "A"]}.get(c, [str(i) for i in range(c)])


def _attr(name: str, typ: str, payload: bytes) -> bytes:
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(payload)) + payload


def _zip_encode(raw: bytes) -> bytes:
    """OpenEXR ZIP: split bytes into even/odd halves, delta-predict, deflate."""
    a = np.frombuffer(raw, dtype=np.uint8)
    t = np.concatenate([a[0::2], a[1::2]])
    d = t.astype(np.int16)
    d[1:] = (t[1:].astype(np.int16) - t[:-1].astype(np.int16) + 128 + 256) % 256
    return zlib.compress(d.astype(np.uint8).tobytes())


def _zip_decode(data: bytes, size: int) -> bytes:
    t = np.frombuffer(zlib.decompress(data), dtype=np.uint8)
    if t.size != size:
        raise ValueError("EXR: corrupt ZIP block")
    d = t.astype(np.int64)
    d[1:] -= 128
    t = (np.cumsum(d) & 0xFF).astype(np.uint8)
    half = (size + 1) // 2
    out = np.empty(size, dtype=np.uint8)
    out[0::2] = t[:half]
    out[1::2] = t[half:]
    return out.tobytes()


def _rle_decode(data: bytes, size: int) -> bytes:
    src = np.frombuffer(data, dtype=np.int8)
    out = bytearray()
    i = 0
    while i < src.size:
        n = int(src[i])
        i += 1
        if n < 0:  # -n literal bytes
            out += src[i:i - n].tobytes()
            i -= n
        else:      # n + 1 copies of the next byte
            out += bytes([src[i] & 0xFF]) * (n + 1)
            i += 1
    if len(out) != size:
        raise ValueError("EXR: corrupt RLE block")
    # the RLE predictor and interleave are the same as ZIP's
    t = np.frombuffer(bytes(out), dtype=np.uint8).astype(np.int64)
    t[1:] -= 128
    t = (np.cumsum(t) & 0xFF).astype(np.uint8)
    half = (size + 1) // 2
    o = np.empty(size, dtype=np.uint8)
    o[0::2] = t[:half]
    o[1::2] = t[half:]
    return o.tobytes()


def write_exr(path: str, img, names=None, compression: int = ZIP_COMPRESSION) -> None:
    """Writes a float32 image [h, w] or [h, w, c] (Bitmap.write of a TensorXf, utils.py:29-46)."""
    a = np.asarray(img, dtype=np.float32)
    if a.ndim == 2:
        a = a[..., None]
    if a.ndim != 3:
        raise ValueError("Invalid image shape")
    h, w, c = a.shape
    names = list(names) if names is not None else channel_names(c)
    if len(names) != c:
        raise ValueError("one channel name per channel")
    if compression not in (NO_COMPRESSION, ZIPS_COMPRESSION, ZIP_COMPRESSION):
        raise ValueError("write_exr supports NO, ZIPS and ZIP compression")
    order = sorted(range(c), key=lambda i: names[i])  # chlist is sorted by name
    chl = b"".join(names[i].encode() + b"\0" + struct.pack("<iB3xii", _PT_FLOAT, 0, 1, 1) for i in order) + b"\0"
    hdr = b"".join([
        _attr("channels", "chlist", chl),
        _attr("compression", "compression", struct.pack("<B", compression)),
        _attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1)),
        _attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1)),
        _attr("lineOrder", "lineOrder", struct.pack("<B", 0)),
        _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0)),
        _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0)),
        _attr("screenWindowWidth", "float", struct.pack("<f", 1.0)),
    ]) + b"\0"
    lines = _LINES[compression]
    # planar per scanline: for each line, each channel's w values
    planar = np.ascontiguousarray(a[:, :, order].transpose(0, 2, 1)).astype('<f4')
    chunks = []
    for y0 in range(0, h, lines):
        raw = planar[y0:y0 + lines].tobytes()
        if compression != NO_COMPRESSION:
            z = _zip_encode(raw)
            if len(z) < len(raw):
                raw = z
        chunks.append(struct.pack("<ii", y0, len(raw)) + raw)
    start = 8 + len(hdr) + 8 * len(chunks)
    offsets, pos = [], start
    for ch in chunks:
        offsets.append(pos)
        pos += len(ch)
    with open(path, "wb") as f:
        f.write(struct.pack("<ii", MAGIC, 2))
        f.write(hdr)
        f.write(struct.pack(f"<{len(offsets)}Q", *offsets))
        for ch in chunks:
            f.write(ch)


def read_exr(path: str, with_names: bool = False):
    """Reads a single-part scanline EXR into float32 [h, w, c] (channels in the file's order,
    which is sorted by name; Bitmap pixel formats Y / YA / RGB(A) are put back in that order)."""
    with open(path, "rb") as f:
        buf = f.read()
    magic, ver = struct.unpack_from("<ii", buf, 0)
    if magic != MAGIC:
        raise ValueError(f"'{path}' is not an OpenEXR file")
    if ver & 0x200 or ver & 0x1000:
        raise ValueError("EXR: tiled / multi-part files are not supported")
    pos = 8
    attrs = {}
    while buf[pos] != 0:
        e = buf.index(b"\0", pos)
        name = buf[pos:e].decode()
        e2 = buf.index(b"\0", e + 1)
        typ = buf[e + 1:e2].decode()
        (size,) = struct.unpack_from("<i", buf, e2 + 1)
        attrs[name] = (typ, buf[e2 + 5:e2 + 5 + size])
        pos = e2 + 5 + size
    pos += 1
    chl = attrs["channels"][1]
    chans, p = [], 0
    while chl[p] != 0:
        e = chl.index(b"\0", p)
        nm = chl[p:e].decode()
        pt, _, xs, ys = struct.unpack_from("<iB3xii", chl, e + 1)
        if xs != 1 or ys != 1:
            raise ValueError("EXR: subsampled channels are not supported")
        chans.append((nm, pt))
        p = e + 1 + 16
    comp = attrs["compression"][1][0]
    if comp not in _LINES:
        raise ValueError(f"EXR: compression {comp} is not supported (NO, RLE, ZIPS, ZIP)")
    x0, y0, x1, y1 = struct.unpack("<iiii", attrs["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    lines = _LINES[comp]
    nchunks = (h + lines - 1) // lines
    offsets = struct.unpack_from(f"<{nchunks}Q", buf, pos)
    line_bytes = sum(_PT_DTYPE[pt].itemsize for _, pt in chans) * w
    out = np.empty((h, len(chans), w), dtype=np.float32)
    for off in offsets:
        yc, size = struct.unpack_from("<ii", buf, off)
        data = buf[off + 8:off + 8 + size]
        nl = min(lines, y1 + 1 - yc)
        full = nl * line_bytes
        if size < full:
            data = _rle_decode(data, full) if comp == RLE_COMPRESSION else _zip_decode(data, full)
        q = 0
        for ly in range(nl):
            for ci, (_, pt) in enumerate(chans):
                dt = _PT_DTYPE[pt]
                out[yc - y0 + ly, ci] = np.frombuffer(data, dtype=dt, count=w, offset=q).astype(np.float32)
                q += dt.itemsize * w
    names = [n for n, _ in chans]
    img = out.transpose(0, 2, 1)
    # Bitmap order of the standard formats (the file stores channels sorted by name)
    for std in (["Y"], ["Y", "A"], ["R", "G", "B"], ["R", "G", "B", "A"]):
        if sorted(std) == sorted(names):
            idx = [names.index(n) for n in std]
            img, names = img[:, :, idx], std
            break
    img = np.ascontiguousarray(img)
    return (img, names) if with_names else img
