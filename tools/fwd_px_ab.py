"""A/B of the voxel-driven forward variants on config 2 (400^3, 400 angles): one plan per
environment setting (read at plan creation), HIP-event times of the forward call, and each
variant's dose compared with the first one's (bit-identical expected for TVAM_FWD_PX 1 vs 2).
usage: python tools/fwd_px_ab.py [N] ["ENV=V ENV=V" ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd.configs import benchy_index_matched, desc_from_config  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    variants = sys.argv[2:] or ["TVAM_FWD_PX=1", "TVAM_FWD_PX=2"]
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(N * N * N, generator=g) * 0.1).cuda()
    G = (torch.rand((N, N, N), generator=g) * 2 - 1).cuda()
    ref = None
    for v in variants:
        env = dict(kv.split("=", 1) for kv in v.split())
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        proj = Projection(desc_from_config(benchy_index_matched(N=N, angles=N)), "cuda:0")
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k)
            else:
                os.environ[k] = old
        out = proj.forward(x)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            proj.forward(x, out=out)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        ts.sort()
        rec = {"variant": v, "fwd_ms_min": ts[0], "fwd_ms_med": ts[len(ts) // 2]}
        if ref is None:
            ref = out.clone()
        else:
            d = (out - ref).abs()
            rec.update({"identical": bool(torch.equal(out, ref)), "max_abs_diff": float(d.max()),
                        "rel_l2": float(torch.linalg.vector_norm(out - ref) / torch.linalg.vector_norm(ref))})
        print(json.dumps(rec), flush=True)
        proj.close()
        del out


if __name__ == "__main__":
    main()
