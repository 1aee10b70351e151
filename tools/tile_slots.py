"""Per-slot in-tile visit counts of one (tile, slice) workgroup of the per-ray tile kernels, in slot
order (diagnostic build, TVAM_TILE_QUEUE=0).  usage: TVAM_LIB=build_variants/libtvam_tilediag.so
python tools/tile_slots.py CONFIG N ANGLES TILE SLICE OUT.npy"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402
from drtvam_amd.configs import cylindrical_refraction, desc_from_config, square_vial  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402

cfgname, N, na, tile, sl, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
cfg = (square_vial(N=N, angles=N, spp=4, regular_sampling=False) if cfgname == "5n"
       else cylindrical_refraction(N=N, angles=N, spp=4, regular_sampling=False))
a0 = N // 3
d = desc_from_config(cfg, angle_range=(a0, a0 + na))
d.flags |= _abi.FLAG_NO_ZERO_SKIP
d.active_total = N * N * N
n = na * N * N
lib = _abi.load_library()
lib.tvam_tile_diag_slots.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
p = Projection(d, "cuda:0")
assert lib.tvam_tile_diag_slots(tile, sl, None, 0) == 0
buf = (ctypes.c_uint * (1 << 21))()
x = torch.rand(n, generator=torch.Generator().manual_seed(0)).cuda() * 0.1
p.forward(x, None, 4, 1)
torch.cuda.synchronize()
assert lib.tvam_tile_diag_slots(tile, sl, buf, 1 << 21) == 0
v = np.frombuffer(buf, dtype=np.uint32).copy()
nz = np.nonzero(v)[0]
v = v[:nz[-1] + 1] if nz.size else v[:0]  # (slots past the workgroup's last one stay 0)
np.save(out, v)
hit = v[v != 0xffffffff]
print(f"slots {v.size} hits {hit.size} mean {hit.mean():.1f} max {hit.max()}", flush=True)
