"""Per-pixel adjoint / forward differences GPU vs oracle on one angle of BASELINE-size scenes
(diagnostic for the flip protocol).  usage: python tools/diag_parity.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402
from drtvam_amd import _abi  # noqa: E402
from drtvam_amd.configs import cylindrical_refraction, cylindrical_scattering, desc_from_config, square_vial  # noqa
from drtvam_amd.engine import Projection  # noqa: E402

OCC = os.path.join(ROOT, "tests", "golden", "occlusion.ply")
DEV = "cuda:0"


def run(name, cfg, N, a0, spp, seed=4, flags=0):
    t0 = time.time()
    d = desc_from_config(cfg, angle_range=(a0, a0 + 1))
    d.flags |= flags
    dfull = desc_from_config(cfg)
    dfull.flags |= flags
    n = N * N
    rng = np.random.default_rng(seed)
    pat = rng.uniform(0.0, 0.1, n).astype(np.float32)
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    pix = (a0 * N * N + np.arange(n)).astype(np.uint32)
    proj = Projection(d, DEV)
    g = proj.adjoint(torch.as_tensor(G, device=DEV), n, None, spp, seed).cpu().numpy().astype(np.float64)
    gref, _ = oracle.adjoint(dfull, G, active_pixels=pix, spp=spp, seed=seed, nthreads=16)
    got = proj.forward(torch.as_tensor(pat, device=DEV), None, spp, seed).cpu().numpy()[..., 0].astype(np.float64)
    ref, _ = oracle.forward(dfull, pat, active_pixels=pix, spp=spp, seed=seed, nthreads=16)
    diff = np.abs(g - gref)
    rel = diff / (np.abs(gref) + 1e-6 * np.abs(gref).max())
    qs = np.quantile(rel, [0.5, 0.9, 0.99, 0.999, 1.0])
    e2 = diff ** 2
    order = np.argsort(-e2)
    top = order[:10]
    share = [float(e2[order[:k]].sum() / e2.sum()) for k in (10, 100, 1000)]
    print(f"{name}: adj rel-L2 {np.linalg.norm(g - gref) / np.linalg.norm(gref):.3e}  fwd rel-L2 "
          f"{np.linalg.norm(got - ref) / np.linalg.norm(ref):.3e}  per-pixel rel quantiles(50/90/99/99.9/max) "
          f"{' '.join(f'{q:.1e}' for q in qs)}  L2 share of top 10/100/1000 pixels {share}  ({time.time() - t0:.0f}s)",
          flush=True)
    for i in top[:5]:
        print(f"    pixel row {i // N} col {i % N}: g {g[i]:.6e} ref {gref[i]:.6e}", flush=True)
    # forward: where is the error
    fd = np.abs(got - ref)
    zi, yi, xi = np.unravel_index(np.argmax(fd), fd.shape)
    print(f"    fwd worst voxel z{zi} y{yi} x{xi}: {got[zi, yi, xi]:.6e} vs {ref[zi, yi, xi]:.6e}; "
          f"per-slice rel err max {np.max(np.linalg.norm((got - ref).reshape(N, -1), axis=1) / (np.linalg.norm(ref.reshape(N, -1), axis=1) + 1e-30)):.2e}",
          flush=True)
    proj.close()


def main():
    which = sys.argv[1:] or ["sq"]
    if "sq" in which:
        for N in (200, 800):
            a0 = int(N * 0.364)
            run(f"square regular N{N}", square_vial(N=N, angles=N), N, a0, 1)
            run(f"square jitter4 N{N}", square_vial(N=N, angles=N, regular_sampling=False, spp=4), N, a0, 4)
            run(f"square jitter4+occ N{N}", square_vial(N=N, angles=N, regular_sampling=False, spp=4,
                                                       occluders=(OCC,)), N, a0, 4)
    if "cyl" in which:
        N = 400
        run("cyl jitter16 albedo0 N400", cylindrical_refraction(N=N, angles=N, regular_sampling=False, spp=16), N, 137, 16)
        run("cyl scatter16 N400", cylindrical_scattering(N=N, angles=N), N, 137, 16)


if __name__ == "__main__":
    main()
