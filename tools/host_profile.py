"""Host-side (Python) cost of the config-2 optimiser iteration: cProfile over N iterations after the
bench's warmup (GPU work overlaps; what the host spends between launches is what shows).

usage: python tools/host_profile.py [N]
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from drtvam_amd import _abi
    from drtvam_amd.optimize import TvamProblem
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfg = bench.scene_config(2, 400, 400)
    cfg["tile"] = 0
    cfg["shard"] = "auto"
    cfg["flags"] = _abi.FLAG_NO_ZERO_SKIP
    dev = torch.device("cuda", 0)
    prob = TvamProblem(cfg, device=dev)
    g = torch.Generator().manual_seed(0)
    prob.x0 = prob.local_from_global(torch.rand(prob.n_global, generator=g) * 0.1)
    for i in range(4):
        prob.iteration(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(4, 4 + n):
        prob.iteration(i)
    torch.cuda.synchronize()
    print(f"plain: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per iteration")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(4 + n, 4 + 2 * n):
        prob.iteration(i)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
