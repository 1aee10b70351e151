"""GPU, two ranks on the one GPU of the box (gloo process group on CUDA
tensors): the sharded optimisation loop with the real HIP projections (planar
path) and the fused L-BFGS (one all-reduce of the dot vector per step) must
reproduce the single-rank run.  Each rank owns a contiguous angle block and
renders a partial dose that is all-reduced; under jittered
sampling (per-ray tile kernels) the forward runs in 4 slice ranges whose async
all-reduces overlap the next range's forward.  A scattering resin (config 4's path loop,
volume.py:179-272) runs its later segments through the brick bins in several chunks per rank
(TVAM_BIN_CHUNK_SLOTS), each rank with its own bin cache, sampler streams by active-set position
(active_base / active_total) and the derived adjoint seed (optimize.py:294-315)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(N=24, angles=12)


SCATTER_CHUNK_SLOTS = 12000  # ~7 chunks for the whole set, ~4 per rank of two


def _run(rank, world, steps, shard):
    from drtvam_amd.configs import benchy_index_matched, cylindrical_scattering
    from drtvam_amd.optimize import TvamProblem

    if shard == "angle_scatter":
        from drtvam_amd import _abi
        cfg = cylindrical_scattering(**CFG, spp=4)
        cfg["shard"] = "angle"
        cfg["flags"] = _abi.FLAG_NO_ZERO_SKIP  # every path marched: the forward bin cache serves the line search
        prob = TvamProblem(cfg, device=torch.device("cuda", 0), rank=rank, world_size=world)
        assert prob.shard == "angle" and prob.proj.desc.albedo == 0.5
        g = torch.Generator().manual_seed(0)
        prob.x0 = prob.local_from_global(torch.rand(prob.n_global, generator=g) * 0.1)
        for i in range(steps):
            prob.iteration(i)
        st = prob.proj.bin_stats()  # the last (line-search) forward's chunks: >= 2, served from this rank's cache
        assert st["chunks"] >= 2 and st["cached"] == st["chunks"], st
        x = prob.gather_patterns(prob.patterns_local().float())
        dose = prob.forward(prob.patterns_local().float().contiguous(), 5)  # all-reduced forward of a new seed
        return np.asarray(prob.loss_hist), x.cpu().numpy(), dose.cpu().numpy()

    jitter = shard == "angle_jitter"  # the per-ray tile path: the dose all-reduce in 4 overlapped slice ranges
    cfg = benchy_index_matched(**CFG, regular_sampling=not jitter, spp=2 if jitter else 1)
    shard = "angle" if jitter else shard
    cfg["shard"] = shard
    prob = TvamProblem(cfg, device=torch.device("cuda", 0), rank=rank, world_size=world)
    assert prob.shard == shard
    g = torch.Generator().manual_seed(0)
    prob.x0 = prob.local_from_global(torch.rand(prob.n_global, generator=g) * 0.1)
    assert prob.proj.planar != jitter
    if jitter and world > 1:
        assert prob.forward_chunks() is not None and len(prob.forward_chunks()) == 4
    for i in range(steps):
        prob.iteration(i)
    x = prob.gather_patterns(prob.patterns_local().float())
    dose = prob.final_render(spp=1)
    return np.asarray(prob.loss_hist), x.cpu().numpy(), dose.cpu().numpy()


def _worker(rank, world, port, steps, shard, q):
    if shard == "angle_scatter":
        os.environ["TVAM_EXPERIMENTAL"] = "1"
        os.environ["TVAM_BIN_CHUNK_SLOTS"] = str(SCATTER_CHUNK_SLOTS)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _run(rank, world, steps, shard)
        if rank == 0:
            q.put(res)
    except BaseException as e:  # report instead of leaving the parent waiting
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("shard", ["slab", "angle", "angle_jitter", "angle_scatter"])
def test_two_rank_gpu_loop_matches_single_rank(shard):
    steps = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()

    def result(procs):
        try:
            res = q.get(timeout=240)
        finally:
            for p in procs:
                p.join(timeout=60)
                if p.is_alive():
                    p.kill()
        assert not (isinstance(res[0], str) and res[0] == "error"), res[2]
        assert all(p.exitcode == 0 for p in procs)
        return res

    p1 = ctx.Process(target=_worker, args=(0, 1, _free_port(), steps, shard, q))
    p1.start()
    ref_loss, ref_x, ref_dose = result([p1])
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, steps, shard, q)) for r in range(2)]
    for p in procs:
        p.start()
    loss, x, dose = result(procs)
    assert ref_loss[-1] < ref_loss[0]
    # the same sums in a different order (partial doses / slab losses): fp32 rounding only
    np.testing.assert_allclose(loss, ref_loss, rtol=1e-4)
    np.testing.assert_allclose(x, ref_x, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(dose, ref_dose, rtol=1e-3, atol=1e-6)
