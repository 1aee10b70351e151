"""Diagnostic of tests/test_gpu_bin_chunks.py's config-4 shard (GPU box): where the subset adjoint
differs from the oracle -- per angle, per chunk, one chunk vs many, first segment vs the rest.
usage: python tools/diag_chunks.py [a0] [n_angles] [stride]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle  # noqa: E402
from drtvam_amd.configs import cylindrical_scattering, desc_from_config  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402
from parity_util import flipped_pixels, rel_l2  # noqa: E402

DEV = "cuda:0"
N, SPP, SEED = 400, 16, 3
a0 = int(sys.argv[1]) if len(sys.argv) > 1 else 120
na = int(sys.argv[2]) if len(sys.argv) > 2 else 20
stride = int(sys.argv[3]) if len(sys.argv) > 3 else 53
oracle.build()
cfg = cylindrical_scattering(N=N, angles=N)
per = N * N
d = desc_from_config(cfg, angle_range=(a0, a0 + na))
dfull = desc_from_config(cfg)
d.active_total = dfull.active_total = N * per
n = na * per
sub = np.arange(0, n, stride, dtype=np.int64)
pix = (a0 * per + sub).astype(np.uint32)
pos = (a0 * per + sub).astype(np.uint64)
rng = np.random.default_rng(7)
G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
gref, _ = oracle.adjoint(dfull, G, active_pixels=pix, spp=SPP, seed=SEED, nthreads=16, streams=pos)
gabs, _ = oracle.adjoint(dfull, np.abs(G), active_pixels=pix, spp=SPP, seed=SEED, nthreads=16, streams=pos)
Gt = torch.as_tensor(G, device=DEV)
proj = Projection(d, DEV)
g = proj.adjoint(Gt, n, None, SPP, SEED).cpu().numpy()
print("bin stats", proj.bin_stats())
os.environ["TVAM_BIN_CHUNK_SLOTS"] = str(1 << 30)
g1 = proj.adjoint(Gt, n, None, SPP, SEED).cpu().numpy()
print("one chunk stats", proj.bin_stats(), "many vs one chunk rel", rel_l2(g, g1), "equal", np.array_equal(g, g1))
del os.environ["TVAM_BIN_CHUNK_SLOTS"]
gs = g[sub]
flip = flipped_pixels(gs, gref, gabs)
keep = ~flip
print(f"subset {sub.size}, flipped {int(flip.sum())}, rel-L2 kept {rel_l2(gs[keep], gref[keep]):.3e}")
r = np.abs(gs - gref) / (gabs + 1e-30)
for q in (0.5, 0.9, 0.99, 0.999, 0.9999):
    print(f"  |g-gref|/gabs quantile {q}: {np.quantile(r[keep], q):.3e}")
ang = sub // per
for a in range(na):
    m = keep & (ang == a)
    print(f"angle {a0 + a}: rel-L2 {rel_l2(gs[m], gref[m]):.3e}  max r {r[m].max():.3e}  n {m.sum()}")
order = np.argsort(-np.abs(gs - gref) * keep)
for i in order[:15]:
    print(f"pixel local {sub[i]} angle {a0 + sub[i] // per} row {(sub[i] % per) // N} col {sub[i] % N}: "
          f"g {gs[i]:.6e} ref {gref[i]:.6e} abs {gabs[i]:.6e} r {r[i]:.3e}")
# the first segments alone (albedo 0 scene: same rays, no scattered part)
d0 = desc_from_config(cfg, angle_range=(a0, a0 + na))
d0.albedo = 0.0
d0f = desc_from_config(cfg)
d0f.albedo = 0.0
d0.active_total = d0f.active_total = N * per
p0 = Projection(d0, DEV)
h = p0.adjoint(Gt, n, None, SPP, SEED).cpu().numpy()[sub]
href, _ = oracle.adjoint(d0f, G, active_pixels=pix, spp=SPP, seed=SEED, nthreads=16, streams=pos)
print(f"albedo 0 (first segments only): rel-L2 {rel_l2(h, href):.3e}")
