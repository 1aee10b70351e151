"""Forward + adjoint of a BASELINE config on an angle shard, for rocprofv3 counter passes.
usage: python tools/profile_jitter.py CONFIG N ANGLES_IN_SHARD [reps]
CONFIG 2: index matched; 3: cylindrical vial (regular sampling, planar kernels); 4: cylindrical
scattering (16 spp); 4a: its first segments only (albedo 0); 5: square vial + occluder (4 spp)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402
from drtvam_amd.configs import (benchy_index_matched, cylindrical_refraction, cylindrical_scattering,  # noqa: E402
                                desc_from_config, square_occluded)
from drtvam_amd.engine import Projection  # noqa: E402


def main():
    cfgname, N, na = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    if cfgname == "5":
        cfg = square_occluded(N=N, angles=N)
    elif cfgname == "2":
        cfg = benchy_index_matched(N=N, angles=N)
    elif cfgname == "3":
        cfg = cylindrical_refraction(N=N, angles=N)
    else:  # "4": config 4; "4a": its first segments only (albedo 0)
        cfg = cylindrical_scattering(N=N, angles=N)
        if cfgname == "4a":
            cfg["vial"]["medium"]["albedo"] = 0.0
    spp = cfg["spp"]
    a0 = N // 3
    d = desc_from_config(cfg, angle_range=(a0, a0 + na), tile=int(os.environ.get("PJ_TILE", "0")))
    d.flags |= _abi.FLAG_NO_ZERO_SKIP
    d.active_total = N * N * N
    n = na * N * N
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(n, generator=g) * 0.1).cuda()
    G = (torch.rand((N, N, N), generator=g) * 2 - 1).cuda()
    t0 = time.perf_counter()
    p = Projection(d, "cuda:0")
    torch.cuda.synchronize()
    print(f"plan {time.perf_counter() - t0:.1f}s", flush=True)
    H = p.count_visits(spp, 0)
    for r in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        p.forward(x, None, spp, 1 + r)
        e.record()
        torch.cuda.synchronize()
        tf = s.elapsed_time(e)
        s.record()
        p.adjoint(G, n, None, spp, 2 + r)
        e.record()
        torch.cuda.synchronize()
        ta = s.elapsed_time(e)
        print(f"config {cfgname} N={N} angles {na}: visits {H:.4e}  fwd {tf:.1f} ms ({H / tf / 1e6:.0f} Gvis/s)  "
              f"adj {ta:.1f} ms ({H / ta / 1e6:.0f} Gvis/s)", flush=True)


if __name__ == "__main__":
    main()
