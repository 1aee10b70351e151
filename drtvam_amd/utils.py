"""Target discretisation and reporting helpers (mirror of drtvam/utils.py).

``discretize`` (utils.py:83-128) voxelises the target mesh into a binary
occupancy grid [Z, Y, X, 1] on the sensor's voxel centres.  The reference casts
one random ray per voxel centre with Mitsuba and tests the hit normal; here the
same inside/outside predicate is evaluated by a scanline parity test along +z
(exact for closed meshes), in numpy.
"""
from __future__ import annotations

import os
import struct

import numpy as np
import torch


def iou_loss(pred, target, threshold=0.9):
    """Intersection over union of (pred > threshold) and (target > 0) (utils.py:8-11)."""
    pred = torch.as_tensor(pred).reshape(-1)
    target = torch.as_tensor(target).reshape(-1)
    obj = target > 0.
    th = pred > threshold
    union = torch.count_nonzero(th | obj)
    return float(torch.count_nonzero(th & obj)) / float(union) if union else 0.0


# ---------------------------------------------------------------------------
# PLY
# ---------------------------------------------------------------------------
_PLY_TYPES = {'char': 'b', 'uchar': 'B', 'short': 'h', 'ushort': 'H', 'int': 'i', 'uint': 'I', 'float': 'f',
              'double': 'd', 'int8': 'b', 'uint8': 'B', 'int16': 'h', 'uint16': 'H', 'int32': 'i', 'uint32': 'I',
              'float32': 'f', 'float64': 'd'}


def read_ply(filename):
    """Vertices (N,3) float64 and triangles (M,3) int64 of a PLY file (ascii or binary_little_endian)."""
    with open(filename, 'rb') as f:
        if f.readline().strip() != b'ply':
            raise ValueError(f"{filename}: not a PLY file")
        fmt = None
        elements = []
        while True:
            line = f.readline().decode('ascii').strip()
            if line.startswith('format'):
                fmt = line.split()[1]
            elif line.startswith('element'):
                _, name, count = line.split()
                elements.append([name, int(count), []])
            elif line.startswith('property'):
                elements[-1][2].append(line.split()[1:])
            elif line == 'end_header':
                break
        data = f.read()
    verts, faces = None, []
    if fmt == 'ascii':
        tokens = data.decode('ascii').split()
        pos = 0
        for name, count, props in elements:
            if name == 'vertex':
                nprop = len(props)
                arr = np.array(tokens[pos:pos + count * nprop], dtype=np.float64).reshape(count, nprop)
                names = [p[-1] for p in props]
                verts = arr[:, [names.index('x'), names.index('y'), names.index('z')]]
                pos += count * nprop
            elif name == 'face':
                for _ in range(count):
                    n = int(tokens[pos])
                    faces.append([int(t) for t in tokens[pos + 1:pos + 1 + n]])
                    pos += 1 + n
            else:
                pos += count * len(props)
    elif fmt == 'binary_little_endian':
        off = 0
        for name, count, props in elements:
            if name == 'vertex' and all(p[0] != 'list' for p in props):
                dt = np.dtype([(p[-1], '<' + _PLY_TYPES[p[0]]) for p in props])
                arr = np.frombuffer(data, dtype=dt, count=count, offset=off)
                off += dt.itemsize * count
                verts = np.stack([arr['x'], arr['y'], arr['z']], axis=1).astype(np.float64)
            elif name == 'face':
                lp = props[0]
                ct, it = '<' + _PLY_TYPES[lp[1]], '<' + _PLY_TYPES[lp[2]]
                cs, isz = struct.calcsize(ct), struct.calcsize(it)
                for _ in range(count):
                    n = struct.unpack_from(ct, data, off)[0]
                    off += cs
                    faces.append(list(struct.unpack_from('<' + _PLY_TYPES[lp[2]] * n, data, off)))
                    off += isz * n
            else:
                dt = np.dtype([(p[-1], '<' + _PLY_TYPES[p[0]]) for p in props])
                off += dt.itemsize * count
    else:
        raise ValueError(f"{filename}: unsupported PLY format {fmt}")
    tris = []
    for fc in faces:
        for i in range(1, len(fc) - 1):
            tris.append([fc[0], fc[i], fc[i + 1]])
    return verts, np.asarray(tris, dtype=np.int64)


def mesh_bbox(filename):
    v, _ = read_ply(filename)
    return v.min(axis=0), v.max(axis=0)


def target_transform(bbox_min, bbox_max, size=1.0, center=(0., 0., 0.)):
    """optimize.py:38-50: centre the mesh bbox, scale its largest extent to `size`, move to `center`."""
    c = 0.5 * (np.asarray(bbox_min) + np.asarray(bbox_max))
    s = size / np.max(np.asarray(bbox_max) - np.asarray(bbox_min))
    m = np.eye(4)
    m[:3, :3] *= s
    m[:3, 3] = np.asarray(center) - s * c
    return m


def voxelize_mesh(verts, tris, bbox_min, voxel_size, res):
    """Binary occupancy [Z, Y, X] of voxel centres inside a closed triangle mesh (z-scanline parity)."""
    rx, ry, rz = res
    xs = bbox_min[0] + (0.5 + np.arange(rx)) * voxel_size[0]
    ys = bbox_min[1] + (0.5 + np.arange(ry)) * voxel_size[1]
    zs = bbox_min[2] + (0.5 + np.arange(rz)) * voxel_size[2]
    occ = np.zeros((rz, ry, rx), dtype=np.uint8)
    a, b, c = verts[tris[:, 0]], verts[tris[:, 1]], verts[tris[:, 2]]
    X, Y = np.meshgrid(xs, ys, indexing='xy')  # [ry, rx]
    # tiny irrational shift of the scan lines: voxel centres of grid-aligned meshes would otherwise
    # pass exactly through shared triangle edges and break the crossing parity
    px = X.reshape(-1) + voxel_size[0] * 1.2345679e-4 * np.sqrt(2.0)
    py = Y.reshape(-1) + voxel_size[1] * 2.3456789e-4 * np.sqrt(3.0)
    crossings = [[] for _ in range(px.size)]
    for t in range(tris.shape[0]):
        A, B, C = a[t], b[t], c[t]
        det = (B[0] - A[0]) * (C[1] - A[1]) - (C[0] - A[0]) * (B[1] - A[1])
        if det == 0:
            continue
        lo = max(np.searchsorted(xs, min(A[0], B[0], C[0])) - 1, 0)
        hi = np.searchsorted(xs, max(A[0], B[0], C[0]), side='right') + 1
        jlo = max(np.searchsorted(ys, min(A[1], B[1], C[1])) - 1, 0)
        jhi = np.searchsorted(ys, max(A[1], B[1], C[1]), side='right') + 1
        if lo >= hi or jlo >= jhi:
            continue
        jj, ii = np.meshgrid(np.arange(jlo, jhi), np.arange(lo, hi), indexing='ij')
        idx = (jj * rx + ii).reshape(-1)
        qx, qy = px[idx], py[idx]
        w1 = ((qx - A[0]) * (C[1] - A[1]) - (C[0] - A[0]) * (qy - A[1])) / det
        w2 = ((B[0] - A[0]) * (qy - A[1]) - (qx - A[0]) * (B[1] - A[1])) / det
        w0 = 1.0 - w1 - w2
        inside = (w0 >= 0) & (w1 >= 0) & (w2 >= 0)
        zc = w0 * A[2] + w1 * B[2] + w2 * C[2]
        for k in np.nonzero(inside)[0]:
            crossings[idx[k]].append(zc[k])
    for p, zl in enumerate(crossings):
        if len(zl) < 2:
            continue
        zl = np.sort(np.asarray(zl))
        j, i = divmod(p, rx)
        for s in range(0, len(zl) - 1, 2):
            m = (zs > zl[s]) & (zs < zl[s + 1])
            occ[m, j, i] = 1
    return occ


def target_triangles(scene):
    """World-space triangles [n, 3, 3] (float32) of the scene's target mesh (optimize.py:30-65)."""
    tgt = scene.target
    if tgt is None or 'filename' not in tgt:
        raise ValueError("No target shape found in the scene")
    verts, tris = read_ply(tgt['filename'])
    m = np.asarray(tgt.get('to_world', np.eye(4)), dtype=np.float64)
    verts = (verts @ m[:3, :3].T + m[:3, 3]).astype(np.float32)
    return verts[np.asarray(tris)]


def discretize(scene, sensor=0):
    """Binary target occupancy [Z, Y, X, 1] float32 on the sensor grid (utils.py:83-128)."""
    if isinstance(sensor, int):
        sensor = scene.sensors()[sensor]
    tgt = scene.target
    if tgt is None:
        raise ValueError("No target shape found in the scene")
    verts, tris = read_ply(tgt['filename'])
    m = np.asarray(tgt.get('to_world', np.eye(4)), dtype=np.float64)
    verts = verts @ m[:3, :3].T + m[:3, 3]
    occ = voxelize_mesh(verts, tris, sensor.bbox_min.astype(np.float64), sensor.voxel_size.astype(np.float64),
                        sensor.resolution())
    return torch.from_numpy(occ.astype(np.float32)[..., None])


def analytic_target(res, bbox_min, bbox_max, kind='box_hole'):
    """Synthetic binary target [Z, Y, X, 1] (used when no mesh file is available).

    'box_hole': box over 80% of x/y and 80% of z with a cylindrical hole of
    radius 20% along z, shifted towards -x (the shape of tests/files/box_hole.ply
    as checked in test_optimization.py:130-144); 'sphere': centred ball.
    """
    rx, ry, rz = res
    bmin, bmax = np.asarray(bbox_min, float), np.asarray(bbox_max, float)
    h = (bmax - bmin) / np.array([rx, ry, rz])
    x = bmin[0] + (0.5 + np.arange(rx)) * h[0]
    y = bmin[1] + (0.5 + np.arange(ry)) * h[1]
    z = bmin[2] + (0.5 + np.arange(rz)) * h[2]
    ext = bmax - bmin
    # broadcast [Z, 1, 1] / [1, Y, 1] / [1, 1, X] (no full-size coordinate grids at 800^3)
    u = ((x - bmin[0]) / ext[0])[None, None, :]
    v = ((y - bmin[1]) / ext[1])[None, :, None]
    w = ((z - bmin[2]) / ext[2])[:, None, None]
    if kind == 'sphere':
        occ = (u - 0.5) ** 2 + (v - 0.5) ** 2 + (w - 0.5) ** 2 < 0.4 ** 2
    else:
        box = (u > 0.1) & (u < 0.9) & (v > 0.1) & (v < 0.9) & (w > 0.1) & (w < 0.9)
        hole = (u - 0.3) ** 2 + (v - 0.5) ** 2 < 0.2 ** 2
        occ = box & ~hole
    return torch.from_numpy(occ.astype(np.float32)[..., None])


def reshape_grid(array):
    """Tiles a stack [n, h, w(, c)] into one square mosaic [rows*h, rows*w, c] (utils.py:13-27)."""
    if len(array.shape) == 3:
        n, h, w = array.shape
        c = 1
    elif len(array.shape) == 4:
        n, h, w, c = array.shape
    else:
        raise ValueError(f"Invalid array shape: {array.shape}")
    rows = int(np.ceil(np.sqrt(n)))
    array_new = np.zeros((rows ** 2, h, w, c))
    array_new[:n] = np.asarray(array).reshape(n, h, w, c)
    return array_new.reshape((rows, rows, h, w, c)).swapaxes(1, 2).reshape((rows * h, rows * w, c))


def save_img(img, path):
    """One image [h, w] or [h, w, c] as an EXR (utils.py:29-37, Bitmap.write)."""
    from .exr import write_exr
    if isinstance(img, torch.Tensor):
        img = img.detach().cpu().numpy()
    img = np.asarray(img, dtype=np.float32)
    if img.ndim not in (2, 3):
        raise ValueError("Invalid image shape")
    write_exr(path, img)


def save_vol(vol, path):
    """A volume [Z, Y, X(, C)] as an EXR mosaic of its slices (utils.py:39-46)."""
    from .exr import write_exr
    if isinstance(vol, torch.Tensor):
        vol = vol.detach().cpu().numpy()
    elif not isinstance(vol, np.ndarray):
        raise ValueError(f"Invalid volume type: '{type(vol)}'")
    write_exr(path, reshape_grid(vol).astype(np.float32))
