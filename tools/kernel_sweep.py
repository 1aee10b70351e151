"""Times the forward / adjoint tile kernels of config 2 for several tile sizes
(HIP events on the launch stream).  Usage: python tools/kernel_sweep.py [N] [tiles...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402
from drtvam_amd.configs import benchy_index_matched, desc_from_config  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402


def bench(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return min(ts), sum(ts) / len(ts)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    tiles = [int(t) for t in sys.argv[2:]] or [0]
    n = N * N * N
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(n, generator=g) * 0.1).cuda()
    G = (torch.rand((N, N, N), generator=g) * 2 - 1).cuda()
    out = torch.empty((N, N, N, 1), device="cuda")
    gout = torch.empty(n, device="cuda")
    for t in tiles:
        d = desc_from_config(benchy_index_matched(N=N, angles=N), tile=t)
        d.flags = _abi.FLAG_NO_ZERO_SKIP
        p = Projection(d, "cuda:0")
        t0 = time.perf_counter()
        H = p.count_visits(1, 0)
        tc = time.perf_counter() - t0
        f = bench(lambda: p.forward(x, None, 1, 0, out=out))
        a = bench(lambda: p.adjoint(G, n, None, 1, 0, out=gout))
        print(f"N={N} tile={t}: visits {H:.4e} (count {tc*1e3:.0f} ms)  fwd min {f[0]:.2f} avg {f[1]:.2f} ms "
              f"({H / f[0] / 1e6:.0f} Gvis/s)  adj min {a[0]:.2f} avg {a[1]:.2f} ms ({H / a[0] / 1e6:.0f} Gvis/s)",
              flush=True)
        p.close()


if __name__ == "__main__":
    main()
