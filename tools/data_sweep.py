"""Forward kernel time vs pattern-value distribution (config 2 geometry)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402
from drtvam_amd.configs import benchy_index_matched, desc_from_config  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402
from tools.kernel_sweep import bench  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    n = N ** 3
    g = torch.Generator().manual_seed(0)
    u = torch.rand(n, generator=g)
    data = {
        "U[0,0.1)": u * 0.1,
        "-U[0,0.1)": -u * 0.1,
        "U[-1,1)": u * 2 - 1,
        "lognormal(0,3)": torch.exp(torch.randn(n, generator=g) * 3),
        "U*1e-30": u * 1e-30,
        "zeros": torch.zeros(n),
    }
    d = desc_from_config(benchy_index_matched(N=N, angles=N))
    d.flags = _abi.FLAG_NO_ZERO_SKIP | _abi.FLAG_FWD_STATS
    p = Projection(d, "cuda:0")
    out = torch.empty((N, N, N, 1), device="cuda")
    for name, x in data.items():
        x = x.cuda().contiguous()
        f = bench(lambda: p.forward(x, None, 1, 0, out=out))
        print(f"{name:16s} fwd min {f[0]:.2f} avg {f[1]:.2f} ms, fallback tiles {p.fallback_tiles()}", flush=True)


if __name__ == "__main__":
    main()
