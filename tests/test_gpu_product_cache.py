"""GPU: the product optimisation loop (drtvam_amd.optimize's TvamProblem, no flags in the config) on
a scattering resin marches every path, as the reference marches every active pixel
(/root/reference/src/drtvam/projector.py:66-70, common.py:81-82), so the line-search forward of an
iteration (lbfgs.py:240-249: the same seed, the direction's pattern) is served from the forward
brick-bin cache, every chunk of it -- the mode bench.py --config 4 measures."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_scattering_line_search_forward_served_from_the_bin_cache(monkeypatch):
    from drtvam_amd import _abi
    from drtvam_amd.configs import cylindrical_scattering
    from drtvam_amd.optimize import TvamProblem

    monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")

    monkeypatch.setenv("TVAM_BIN_CHUNK_SLOTS", "12000")  # several chunks
    cfg = cylindrical_scattering(N=24, angles=12, spp=4)
    assert "flags" not in cfg
    prob = TvamProblem(cfg, device=torch.device("cuda", 0))
    assert prob.proj.desc.albedo == 0.5
    assert prob.proj.desc.flags & _abi.FLAG_NO_ZERO_SKIP
    g = torch.Generator().manual_seed(0)
    prob.x0 = prob.local_from_global(torch.rand(prob.n_global, generator=g) * 0.1)
    for i in range(3):
        prob.iteration(i)
        st = prob.proj.bin_stats()  # the iteration's last binned call: its line-search forward
        assert st["chunks"] >= 2 and st["cached"] == st["chunks"] and st["count_mismatch"] == 0, (i, st)
    assert np.isfinite(prob.loss_hist).all() and prob.loss_hist[-1] < prob.loss_hist[0]
