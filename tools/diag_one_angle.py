"""Times the GPU calls of tests/test_gpu_baseline_sizes.py::_one_angle (config 4, one angle of 400,
16 spp) step by step with a sync and a line after each, to find a slow or stuck call.
usage: python tools/diag_one_angle.py [config=4]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd.configs import cylindrical_scattering, desc_from_config, square_occluded  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402


def main():
    c = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    N = 400 if c == 4 else 800
    cfg = cylindrical_scattering(N=N, angles=N) if c == 4 else square_occluded(N=N, angles=N)
    a0, spp = (137, 16) if c == 4 else (291, 4)
    d = desc_from_config(cfg, angle_range=(a0, a0 + 1))
    n = N * N
    d.active_total = N * n
    rng = np.random.default_rng(3)
    pat = torch.as_tensor(rng.uniform(0.0, 0.1, n).astype(np.float32), device="cuda:0")
    G = torch.as_tensor(rng.uniform(-1, 1, (N, N, N)).astype(np.float32), device="cuda:0")
    t = time.perf_counter()
    proj = Projection(d, "cuda:0")
    torch.cuda.synchronize()
    print(f"plan {time.perf_counter() - t:.2f}s", flush=True)
    for name, fn in (("adjoint", lambda: proj.adjoint(G, n, None, spp, 3)),
                     ("forward", lambda: proj.forward(pat, None, spp, 3)),
                     ("forward (cached)", lambda: proj.forward(pat, None, spp, 3)),
                     ("adjoint", lambda: proj.adjoint(G, n, None, spp, 3))):
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        print(f"{name} {time.perf_counter() - t:.3f}s sum {float(out.double().sum()):.6e} bins {proj.bin_stats()}",
              flush=True)


if __name__ == "__main__":
    main()
