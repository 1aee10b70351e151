"""GPU: the angle-sharded loop's collectives on RCCL (torch.distributed 'nccl' backend) at world
size 1 on the box's one GPU.  With config 'collectives': 'always' the loop runs every collective of
an N-rank run -- the dose all-reduces (under jittered sampling in 4 slice ranges, each range's async
all-reduce issued before the next range's forward), the L-BFGS dot vector and
the loss all-reduces -- and must reproduce the run without a process group (a sum over one rank).  Reference: /root/reference/src/drtvam/optimize.py:292-320, lbfgs.py:240-249."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _run(kind, steps, with_pg):
    import torch.distributed as dist
    from drtvam_amd.configs import benchy_index_matched
    from drtvam_amd.optimize import TvamProblem

    jitter = kind == "jitter"
    cfg = benchy_index_matched(N=24, angles=12, regular_sampling=not jitter, spp=2 if jitter else 1)
    cfg["shard"] = "angle"
    cfg["collectives"] = "always"
    prob = TvamProblem(cfg, device=torch.device("cuda", 0), rank=0, world_size=1)
    calls = {"all_reduce": 0, "async": 0}
    if with_pg:
        assert prob.dist is not None and dist.get_backend() == "nccl"
        orig = dist.all_reduce

        def counted(t, *a, **kw):
            calls["all_reduce"] += 1
            calls["async"] += int(bool(kw.get("async_op")))
            return orig(t, *a, **kw)

        dist.all_reduce = counted
        if jitter:
            assert prob.forward_chunks() is not None and len(prob.forward_chunks()) == 4
    else:
        assert prob.dist is None
    g = torch.Generator().manual_seed(0)
    prob.x0 = prob.local_from_global(torch.rand(prob.n_global, generator=g) * 0.1)
    for i in range(steps):
        prob.iteration(i)
    x = prob.patterns_local().float()
    torch.cuda.synchronize()
    if with_pg:
        dist.all_reduce = orig
    return np.asarray(prob.loss_hist), x.cpu().numpy(), calls


def _worker(kind, steps, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        try:
            q.put(_run(kind, steps, True))
        finally:
            dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put(("error", traceback.format_exc()))
        raise


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind", ["planar", "jitter"])
def test_rccl_world_size_one_matches_no_process_group(kind):
    steps = 2
    ref_loss, ref_x, _ = _run(kind, steps, False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(kind, steps, _free_port(), q))
    p.start()
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert not (isinstance(res[0], str) and res[0] == "error"), res[1]
    loss, x, calls = res
    assert p.exitcode == 0
    # dose all-reduces (2 per iteration; 4 async slice ranges each under jittered sampling) + the
    # dot vector and the loss per iteration
    assert calls["all_reduce"] >= 2 * steps, calls
    if kind == "jitter":
        assert calls["async"] == 2 * 4 * steps, calls
    # a sum over one rank; the jittered forward's slice ranges re-derive their fixed-point scales
    np.testing.assert_allclose(loss, ref_loss, rtol=1e-6)
    np.testing.assert_allclose(x, ref_x, rtol=1e-5, atol=1e-7)
