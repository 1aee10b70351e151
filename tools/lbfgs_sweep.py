"""Time the fused L-BFGS vector passes at config 2's size (400 angles x 400^2 = 64M patterns,
full history h = 5, a new pair each step) under the current TVAM_VEC_* env knobs.
usage: python tools/lbfgs_sweep.py [n]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400 ** 3
    dev = "cuda:0"
    lib = _abi.load_library()
    stream = torch.cuda.current_stream().cuda_stream
    h = 5
    g = torch.rand(n, device=dev)
    p, p_old, g_old = torch.rand(n, device=dev), torch.rand(n, device=dev), torch.rand(n, device=dev)
    S = torch.rand((h + 1, n), device=dev)
    Y = torch.rand((h + 1, n), device=dev)
    work = torch.empty(_abi.LBFGS_WORK_DOUBLES, dtype=torch.float64, device=dev)
    dots = torch.empty(64, dtype=torch.float64, device=dev)
    d = torch.empty(n, device=dev)
    Sp = (ctypes.c_void_p * h)(*[S[j].data_ptr() for j in range(h)])
    Yp = (ctypes.c_void_p * h)(*[Y[j].data_ptr() for j in range(h)])
    cs = (ctypes.c_float * (h + 1))(*[0.1] * (h + 1))
    cy = (ctypes.c_float * (h + 1))(*[0.2] * (h + 1))
    Sp6 = (ctypes.c_void_p * (h + 1))(*[S[j].data_ptr() for j in range(h + 1)])
    Yp6 = (ctypes.c_void_p * (h + 1))(*[Y[j].data_ptr() for j in range(h + 1)])

    def hist():
        _abi.check(lib.tvam_lbfgs_history(n, p.data_ptr(), p_old.data_ptr(), g.data_ptr(), g_old.data_ptr(), h, Sp, Yp,
                                          S[h].data_ptr(), Y[h].data_ptr(), work.data_ptr(), dots.data_ptr(), stream))

    def direction():
        _abi.check(lib.tvam_lbfgs_direction(n, g.data_ptr(), h + 1, Sp6, Yp6, 0.5, cs, cy, d.data_ptr(), stream))

    def axpy():
        _abi.check(lib.tvam_axpy_clamp(n, p.data_ptr(), 0.01, d.data_ptr(), 0.0, p_old.data_ptr(), stream))

    res = {}
    for name, fn, nbytes in [("hist", hist, 4 * n * (4 + 2 * h + 2)), ("dir", direction, 4 * n * (2 + 2 * (h + 1))),
                             ("axpy", axpy, 4 * n * 3)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        res[name] = {"ms": round(ms, 4), "GB/s": round(nbytes / ms / 1e6, 1)}
    env = {k: v for k, v in os.environ.items() if k.startswith("TVAM_VEC")}
    import hashlib
    hist()
    direction()
    torch.cuda.synchronize()
    res["dots_sha"] = hashlib.sha256(dots.cpu().numpy().tobytes()).hexdigest()[:16]
    res["d_sha"] = hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"env": env, "lib": os.environ.get("TVAM_LIB", ""), **res}))


if __name__ == "__main__":
    main()
