"""Renders single DMD pixels (sparse active set, pattern 1) of a BASELINE-size scene on the GPU and
in the oracle and reports where their doses differ (diagnostic).  usage: python tools/diag_pixel.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402
from drtvam_amd.configs import cylindrical_refraction, desc_from_config, square_vial  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402

DEV = "cuda:0"


def pixel(name, cfg, N, a0, row, col, spp, seed=4):
    d = desc_from_config(cfg)
    proj = Projection(d, DEV)
    pix = np.array([a0 * N * N + row * N + col], dtype=np.uint32)
    one = np.ones(1, dtype=np.float32)
    got = proj.forward(torch.ones(1, device=DEV), torch.as_tensor(pix.astype(np.int32), device=DEV), spp,
                       seed).cpu().numpy()[..., 0].astype(np.float64)
    ref, visits = oracle.forward(d, one, active_pixels=pix, spp=spp, seed=seed, nthreads=1)
    nz_g, nz_r = got != 0, ref != 0
    print(f"{name} a{a0} r{row} c{col}: sum gpu {got.sum():.6e} oracle {ref.sum():.6e}; nonzero voxels gpu "
          f"{int(nz_g.sum())} oracle {int(nz_r.sum())} (oracle visits {visits}); only-gpu {int((nz_g & ~nz_r).sum())} "
          f"only-oracle {int((nz_r & ~nz_g).sum())}", flush=True)
    diff = np.abs(got - ref)
    idx = np.argsort(-diff.ravel())[:6]
    for i in idx:
        z, y, x = np.unravel_index(i, got.shape)
        print(f"    z{z} y{y} x{x}: gpu {got[z, y, x]:.6e} oracle {ref[z, y, x]:.6e}", flush=True)
    zs_g = sorted(set(np.nonzero(nz_g)[0].tolist()))
    zs_r = sorted(set(np.nonzero(nz_r)[0].tolist()))
    print(f"    slices gpu {zs_g} oracle {zs_r}", flush=True)
    # per sample: the oracle ray of each of the spp samples
    for k in range(spp):
        r = oracle.ray(d, int(pix[0]), wave_index=int(pix[0]) * spp + k, seed=seed)
        print(f"    sample {k}: o {np.round(r['o'], 6).tolist()} hit {r.get('hit')} o2 {r.get('o2')} maxt "
              f"{r.get('maxt')}", flush=True)
    proj.close()


def main():
    N = 400
    cyl = cylindrical_refraction(N=N, angles=N, regular_sampling=False, spp=16)
    for row, col in ((300, 307), (250, 351), (222, 293)):
        pixel("cyl jitter16", cyl, N, 137, row, col, 16)
    N = 800
    sq = square_vial(N=N, angles=N, regular_sampling=False, spp=4)
    for row, col in ((628, 684), (555, 579), (410, 566)):
        pixel("square jitter4", sq, N, 291, row, col, 4)


if __name__ == "__main__":
    main()
