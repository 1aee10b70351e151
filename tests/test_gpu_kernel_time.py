"""GPU: the dominant-kernel launch timer that bench.py's live roofline divides by
(tvam_plan_kernel_time): one recorded launch per forward of a voxel-driven planar plan (its
forward kernel, not the slice binning or the adjoint), none while disabled, and times that agree
with the whole forward call's HIP-event time from above."""
import numpy as np
import pytest
import torch

from drtvam_amd.configs import benchy_index_matched, desc_from_config
from drtvam_amd.engine import Projection

pytestmark = pytest.mark.gpu


def test_kernel_time_counts_forward_launches():
    N = 96
    d = desc_from_config(benchy_index_matched(N=N, angles=24))
    p = Projection(d, "cuda:0")
    try:
        assert p.planar_forward
        n = int(d.crop_x) * int(d.crop_y) * 24
        x = torch.as_tensor(np.random.default_rng(3).uniform(0, 1, n).astype(np.float32), device="cuda:0")
        G = torch.rand((N, N, N), device="cuda:0")
        p.forward(x, None, 1, 0)
        torch.cuda.synchronize()
        assert p.kernel_time(False) == (0.0, 0)  # nothing recorded while disabled
        p.kernel_time(True)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            p.forward(x, None, 1, 0)
        e.record()
        p.adjoint(G, n, None, 1, 0)  # not the dominant forward kernel: not recorded
        ms, launches = p.kernel_time(False)
        torch.cuda.synchronize()
        assert launches == 3
        assert 0.0 < ms <= s.elapsed_time(e) * 1.05 + 0.05
        assert p.kernel_time(False) == (0.0, 0)  # stopped
    finally:
        p.close()


def test_kernel_timer_is_owned_by_its_plan():
    """one timer per process, owned by the plan that enabled it: another plan cannot
    take it while it runs; reading it or destroying the owner releases it (and its events)."""
    from drtvam_amd._abi import TvamError
    d = desc_from_config(benchy_index_matched(N=32, angles=8))
    a, b = Projection(d, "cuda:0"), Projection(d, "cuda:0")
    try:
        n = int(d.crop_x) * int(d.crop_y) * 8
        x = torch.rand(n, device="cuda:0")
        a.kernel_time(True)
        with pytest.raises((TvamError, RuntimeError, ValueError)):
            b.kernel_time(True)
        b.forward(x, None, 1, 0)  # the timer records its kernel kind on its device, whichever plan launches
        a.forward(x, None, 1, 0)
        ms, launches = a.kernel_time(False)  # read: released
        assert launches == 2 and ms > 0.0
        b.kernel_time(True)
        b.forward(x, None, 1, 0)
        b.close()  # the owner goes: the timer and its events with it
        b = None
        a.kernel_time(True)
        a.forward(x, None, 1, 0)
        assert a.kernel_time(False)[1] == 1
    finally:
        a.close()
        if b is not None:
            b.close()
