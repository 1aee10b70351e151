"""GPU, two ranks on the one GPU of the box (gloo process group on CUDA
tensors): the sharded optimisation loop with the real HIP projections (planar
path) and the fused L-BFGS (one all-reduce of the dot vector per step) must
reproduce the single-rank run.  Each rank owns a contiguous angle block and
renders a partial dose that is all-reduced."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(N=24, angles=12)


def _run(rank, world, steps):
    from drtvam_amd.configs import benchy_index_matched
    from drtvam_amd.optimize import TvamProblem

    cfg = benchy_index_matched(**CFG)
    prob = TvamProblem(cfg, device=torch.device("cuda", 0), rank=rank, world_size=world)
    g = torch.Generator().manual_seed(0)
    full = torch.rand(prob.n_global, generator=g) * 0.1
    per = prob.n_global // CFG["angles"]
    prob.x0 = full[prob.a0 * per:prob.a1 * per].cuda().contiguous()
    assert prob.proj.planar
    for i in range(steps):
        prob.iteration(i)
    x = prob.patterns_local().float()
    if world > 1:
        sizes = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([x.numel()], device="cuda"))
        m = int(max(int(s) for s in sizes))
        parts = [torch.zeros(m, device="cuda") for _ in range(world)]
        pad = torch.zeros(m, device="cuda")
        pad[:x.numel()] = x
        dist.all_gather(parts, pad)
        x = torch.cat([p[:int(s)] for p, s in zip(parts, sizes)])
    return np.asarray(prob.loss_hist), x.cpu().numpy()


def _worker(rank, world, port, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        loss, x = _run(rank, world, steps)
        if rank == 0:
            q.put((loss, x))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gpu_loop_matches_single_rank():
    steps = 4
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p1 = ctx.Process(target=_worker, args=(0, 1, _free_port(), steps, q))
    p1.start()
    ref_loss, ref_x = q.get()
    p1.join(timeout=300)
    assert p1.exitcode == 0
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    loss, x = q.get()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert ref_loss[-1] < ref_loss[0]
    # partial doses sum in a different order: fp32 rounding only
    np.testing.assert_allclose(loss, ref_loss, rtol=1e-4)
    np.testing.assert_allclose(x, ref_x, rtol=1e-3, atol=1e-5)
