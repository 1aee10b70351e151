"""A/B of projection variants on config 2 (400^3, 400 angles): one plan per variant (environment
read at plan creation; "tile=T" sets desc.tile), HIP-event times of the forward and adjoint calls,
and each variant's dose / gradient compared with the first variant's.
usage: python tools/proj_ab.py [N] ["ENV=V ENV=V tile=T" ...]"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd.configs import benchy_index_matched, desc_from_config  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402


def timed(fn, reps=15):
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
    ts.sort()
    return ts[0], ts[len(ts) // 2]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    variants = sys.argv[2:] or [""]
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(N * N * N, generator=g) * 0.1).cuda()
    G = (torch.rand((N, N, N), generator=g) * 2 - 1).cuda()
    ref = None
    for v in variants:
        kv = dict(t.split("=", 1) for t in v.split())
        tile = int(kv.pop("tile", 0))
        saved = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        proj = Projection(desc_from_config(benchy_index_matched(N=N, angles=N), tile=tile), "cuda:0")
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k)
            else:
                os.environ[k] = old
        dose = proj.forward(x)
        grad = proj.adjoint(G, x.numel())
        fmin, fmed = timed(lambda: proj.forward(x, out=dose))
        amin, amed = timed(lambda: proj.adjoint(G, x.numel(), out=grad))
        rec = {"variant": v, "fwd_ms_min": fmin, "fwd_ms_med": fmed, "adj_ms_min": amin, "adj_ms_med": amed,
               "dose_sha": hashlib.sha256(dose.cpu().numpy().tobytes()).hexdigest()[:16],
               "grad_sha": hashlib.sha256(grad.cpu().numpy().tobytes()).hexdigest()[:16]}
        if ref is None:
            ref = (dose.clone(), grad.clone())
        else:
            for name, a, b in (("dose", dose, ref[0]), ("grad", grad, ref[1])):
                rec[f"{name}_identical"] = bool(torch.equal(a, b))
                rec[f"{name}_rel_l2"] = float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b))
        print(json.dumps(rec), flush=True)
        proj.close()
        del dose, grad


if __name__ == "__main__":
    main()
