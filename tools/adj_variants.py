"""Config-2 planar adjoint under plan-time variants (environment knobs read at plan creation),
HIP-event timed on the launch stream.  usage: python tools/adj_variants.py "K=V,K=V" "K=V" ...
(an empty string = defaults); TVAM_CONFIG=3 for the cylindrical vial."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402
from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402


def main():
    N = 400
    n = N * N * N
    g = torch.Generator().manual_seed(0)
    G = (torch.rand((N, N, N), generator=g) * 2 - 1).cuda()
    gout = torch.empty(n, device="cuda")
    mk = cylindrical_refraction if os.environ.get("TVAM_CONFIG") == "3" else benchy_index_matched
    ref = None
    for var in sys.argv[1:] or [""]:
        kv = dict(x.split("=") for x in var.split(",") if x)
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        d = desc_from_config(mk(N=N, angles=N))
        d.flags = _abi.FLAG_NO_ZERO_SKIP
        p = Projection(d, "cuda:0")
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
        p.adjoint(G, n, None, 1, 0, out=gout)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            p.adjoint(G, n, None, 1, 0, out=gout)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        if ref is None:
            ref = gout.clone()
        err = float(torch.linalg.norm(gout - ref) / torch.linalg.norm(ref))
        print(f"{var or 'defaults':60s} adj min {min(ts):.3f} avg {sum(ts) / len(ts):.3f} ms  rel to first {err:.1e}",
              flush=True)
        p.close()


if __name__ == "__main__":
    main()
