"""Multi-rank path on CPU (gloo, world_size 2): the sharded optimisation loop.

Each rank owns a contiguous block of projector angles (= a block of columns of
the linear projection operator), renders a partial dose that is all-reduced,
back-projects rank-locally and all-reduces every L-BFGS dot.  The sharded run
must reproduce the single-rank run.  The GPU projection
is replaced by a dense CPU operator with the same contract.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from drtvam_amd.loss import ThresholdedLoss
from drtvam_amd.optimize import ShardedLoop, angle_shard

SHAPE = (4, 5, 6, 1)
A, PER_ANGLE = 6, 7


def operator():
    g = torch.Generator().manual_seed(0)
    V = int(np.prod(SHAPE))
    M = torch.rand((V, A * PER_ANGLE), generator=g, dtype=torch.float64) * 0.05
    M[M < 0.03] = 0.0  # sparse-ish, like a projector
    target = (torch.rand(SHAPE, generator=g) > 0.5).to(torch.float64)
    return M, target


class MatrixShard(ShardedLoop):
    def __init__(self, rank, world, chunked=False):
        self.chunked = chunked
        M, target = operator()
        self.a0, self.a1 = angle_shard(A, rank, world)
        self.M = M[:, self.a0 * PER_ANGLE:self.a1 * PER_ANGLE]
        self.dist = dist if world > 1 else None
        self.rank, self.world = rank, world
        self.target = target
        self.loss_fn = ThresholdedLoss({"tl": 0.3, "tu": 0.4})
        self.fused = False
        self.n_global = A * PER_ANGLE
        self.n_local = self.M.shape[1]
        self.x0 = torch.full((self.n_local,), 0.5, dtype=torch.float64)
        self.grad_vol = None
        self.opt = None
        self.loss_hist = []

    def forward_local(self, x, seed):
        return (self.M @ x.detach()).reshape(SHAPE).contiguous()

    def adjoint_local(self, grad_vol, seed):
        return self.M.T @ grad_vol.reshape(-1)

    # slice-range forward: the overlapped chunk-by-chunk dose all-reduce (async gloo here)
    def forward_chunks(self):
        return [(0, 1), (1, 3), (3, 4)] if self.chunked else None

    def forward_local_slices(self, x, seed, z0, z1, out):
        out[z0:z1] = self.forward_local(x, seed)[z0:z1]
        return out

    def dose_buffer(self):
        return torch.empty(SHAPE, dtype=torch.float64)


def run(rank, world, steps, chunked=False):
    prob = MatrixShard(rank, world, chunked)
    for i in range(steps):
        prob.iteration(i)
    x = prob.patterns_local()
    if world > 1:
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x)
        x = torch.cat(parts)
    return np.asarray(prob.loss_hist), x.numpy()


def _worker(rank, world, port, steps, q, chunked=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        loss, x = run(rank, world, steps, chunked)
        if rank == 0:
            q.put((loss, x))
    finally:
        dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_angle_shard_partition():
    for n, w in [(400, 8), (7, 3), (5, 8)]:
        blocks = [angle_shard(n, r, w) for r in range(w)]
        assert blocks[0][0] == 0 and blocks[-1][1] == n
        assert all(b[1] == c[0] for b, c in zip(blocks, blocks[1:]))
        assert max(b[1] - b[0] for b in blocks) - min(b[1] - b[0] for b in blocks) <= 1


@pytest.mark.parametrize("chunked", [False, True])
def test_sharded_loop_matches_single_rank(chunked):
    steps = 6
    ref_loss, ref_x = run(0, 1, steps)
    assert ref_loss[-1] < ref_loss[0]
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, steps, q, chunked)) for r in range(2)]
    for p in procs:
        p.start()
    loss, x = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    np.testing.assert_allclose(loss, ref_loss, rtol=1e-9)
    np.testing.assert_allclose(x, ref_x, rtol=1e-9, atol=1e-12)
