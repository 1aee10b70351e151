"""Time the fused L-BFGS passes at config 2's size (64 M patterns, 5 retained pairs) for one
launch geometry (TVAM_VEC_HGRID / TVAM_VEC_DGRID, read once per process): one JSON line."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402

lib = _abi.load_library()
n, h = 400 * 400 * 400, 4
dev = torch.device("cuda", 0)
V = torch.rand(2 * h + 6, n, device=dev)
S = [V[j] for j in range(h + 1)]
Y = [V[h + 1 + j] for j in range(h + 1)]
p, p_old, g, g_old, d = V[2 * h + 2], V[2 * h + 3], V[2 * h + 4], V[2 * h + 5], torch.empty(n, device=dev)
work = torch.empty(_abi.LBFGS_WORK_DOUBLES, dtype=torch.float64, device=dev)
dots = torch.empty(64, dtype=torch.float64, device=dev)
coef = torch.zeros(17, dtype=torch.float32, device=dev)
coef[:] = 0.1
st = torch.cuda.current_stream().cuda_stream
Sp = (ctypes.c_void_p * 8)(*[s.data_ptr() for s in S])
Yp = (ctypes.c_void_p * 8)(*[y.data_ptr() for y in Y])


def hist():
    _abi.check(lib.tvam_lbfgs_history(n, p.data_ptr(), p_old.data_ptr(), g.data_ptr(), g_old.data_ptr(), h, Sp, Yp,
                                      S[h].data_ptr(), Y[h].data_ptr(), work.data_ptr(), dots.data_ptr(), st))


def direction():
    _abi.check(lib.tvam_lbfgs_direction_dev(n, g.data_ptr(), h + 1, Sp, Yp, coef.data_ptr(), d.data_ptr(), st))


def timed(fn, reps=30):
    for _ in range(3):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for i in range(reps):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
    return t[len(t) // 2]


th, td = timed(hist), timed(direction)
print(json.dumps({"hgrid": os.environ.get("TVAM_VEC_HGRID", "768"), "dgrid": os.environ.get("TVAM_VEC_DGRID", "1024"),
                  "hist_ms": th, "hist_TBps": (2 * h + 6) * n * 4 / th / 1e9,
                  "dir_ms": td, "dir_TBps": (2 * h + 4) * n * 4 / td / 1e9}))
