"""Target discretisation and reporting helpers (mirror of drtvam/utils.py).

``discretize`` (utils.py:83-128) voxelises the target mesh into a binary
occupancy grid [Z, Y, X, 1] on the sensor's voxel centres with the reference's
algorithm (one sampled ray per voxel centre, orientation of the first hit), on
the GPU through ``tvam_discretize``.
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
    """optimize.py:38-50: centre the mesh bbox, scale its largest extent to `size`, move to
    `center`: translate(center) @ scale(size / max(extents)) @ translate(-c), with c, the scale
    and the translation rounded to fp32 as Mitsuba's ScalarTransform4f forms them."""
    f = np.float32
    bmin, bmax = np.asarray(bbox_min, f), np.asarray(bbox_max, f)
    c = f(0.5) * (bmin + bmax)
    s = f(size) / np.max(bmax - bmin)
    t = np.asarray(center, f) + s * (-c)
    m = np.eye(4)
    m[:3, :3] *= float(s)
    m[:3, 3] = t.astype(np.float64)
    return m


def transform_points(m, verts):
    """fp32 world positions of mesh vertices under the affine 4x4 `m` (Mitsuba's
    transform_affine: one fused multiply-add chain per coordinate; products of fp32 values are
    exact in float64, so one float64 sum rounded to fp32 stands in for the fma chain)."""
    m = np.asarray(m, np.float64)
    v = np.asarray(verts, np.float32).astype(np.float64)
    return (v @ m[:3, :3].T + m[:3, 3]).astype(np.float32)


def cuboid_triangles(lo, hi):
    """The 12 outward-facing triangles [12, 3, 3] (float32) of the box [lo, hi]."""
    lo, hi = np.asarray(lo, np.float32), np.asarray(hi, np.float32)
    c = np.array([[(hi if (i >> a) & 1 else lo)[a] for a in range(3)] for i in range(8)], np.float32)
    quads = [(0, 2, 6, 4), (1, 5, 7, 3), (0, 4, 5, 1), (2, 3, 7, 6), (0, 1, 3, 2), (4, 6, 7, 5)]  # -x +x -y +y -z +z
    tris = []
    for q in quads:
        tris += [(q[0], q[1], q[2]), (q[0], q[2], q[3])]
    t = c[np.asarray(tris)]
    inward = np.einsum('ij,ij->i', np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0]),
                       t.mean(axis=1) - 0.5 * (lo + hi)) < 0
    t[inward] = t[inward][:, ::-1]
    return t


def target_triangles(scene):
    """World-space triangles [n, 3, 3] (float32) of the scene's target mesh (optimize.py:30-65).
    An analytic target (no mesh file, analytic_target) is represented by the cuboid that bounds
    its occupied voxels, u, v, w in [0.1, 0.9] of the sensor box: the Radon filter keeps a
    superset of the pixels whose rays cross the shape."""
    tgt = scene.target
    if tgt is not None and tgt.get('type') == 'analytic':
        sensor = scene.sensor_by_id('sensor')
        bmin, bmax = np.asarray(sensor.bbox_min, np.float64), np.asarray(sensor.bbox_max, np.float64)
        return cuboid_triangles(bmin + 0.1 * (bmax - bmin), bmin + 0.9 * (bmax - bmin))
    if tgt is None or 'filename' not in tgt:
        raise ValueError("No target shape found in the scene")
    verts, tris = read_ply(tgt['filename'])
    return transform_points(tgt.get('to_world', np.eye(4)), verts)[np.asarray(tris)]


def discretize(scene, sensor=0):
    """Binary target occupancy [Z, Y, X, 1] float32 on the sensor grid (utils.py:83-128).

    As the reference: one ray per voxel centre, direction square_to_uniform_sphere of the
    independent sampler seeded (0, voxels) at lane = voxel index, inside when the centre lies
    strictly inside the target bbox and the first target hit faces away from the ray
    (dot(n, d) > 0).  Runs on the GPU (`tvam_discretize`); there is no CPU path.
    """
    import ctypes
    from . import _abi
    if isinstance(sensor, int):
        sensor = scene.sensors()[sensor]
    if scene.target is None or 'filename' not in scene.target:
        raise ValueError("No target shape found in the scene")
    if not torch.cuda.is_available():
        raise _abi.TvamError("discretize runs on the GPU (tvam_discretize); no ROCm device is visible")
    d = _abi.default_desc()
    rx, ry, rz = sensor.resolution()
    d.film_res[:] = (rx, ry, rz)
    d.bbox_min[:] = [float(v) for v in sensor.bbox_min]
    d.bbox_max[:] = [float(v) for v in sensor.bbox_max]
    d.set_target(target_triangles(scene))
    dev = torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((rz, ry, rx), dtype=torch.float32, device=dev)
    lib = _abi.load_library()
    _abi.check(lib.tvam_discretize(ctypes.byref(d), out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
    return out.cpu()[..., None]


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
