"""GPU parity of the general per-path kernel: 'ratio' and 'delta' sensors (sensor.py:112-295)
and sample_time (common.py:101-104), against the oracle on identical sampler streams, plus the
reference's own FD-vs-AD test of tests/test_integrators.py:69-110 (dda / ratio / delta on its
double-cylinder scattering scene with sample_time, 128 spp, bar 2e-4).

Tolerance vs the oracle: the flip protocol of parity_util.py, like the scattering tests (host and
device libm may differ in the last ulp of logf / sinf, which can flip a comparison on a rare
path: those paths' pixels are counted, every other path is held to 1e-4 relative L2)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from drtvam_amd import _abi
from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, desc_from_config
from drtvam_amd.engine import Projection, render
from parity_util import flip_protocol


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def make(sensor="dda", albedo=0.0, vial="index_matched", regular=False, spp=2, sample_time=False, N=16, A=8,
         majorant=3.0):
    if vial == "index_matched":
        cfg = benchy_index_matched(N=N, angles=A, size_mm=4.0, r=2.9, sigma_t=0.4, regular_sampling=regular, spp=spp)
    else:
        cfg = cylindrical_refraction(N=N, angles=A, size_mm=4.0, r_int=3.5, r_ext=4.0, sigma_t=0.4,
                                     regular_sampling=regular, spp=spp)
    d = desc_from_config(cfg)
    d.albedo = albedo
    d.phase_type = _abi.PHASE_RAYLEIGH
    d.sensor_type = {"dda": _abi.SENSOR_DDA, "ratio": _abi.SENSOR_RATIO, "delta": _abi.SENSOR_DELTA}[sensor]
    d.majorant = majorant
    d.sample_time = int(sample_time)
    return d


CASES = [
    dict(sensor="ratio"),
    dict(sensor="ratio", albedo=0.5),
    dict(sensor="ratio", albedo=0.5, vial="cylindrical"),
    dict(sensor="delta", albedo=0.5),
    dict(sensor="delta", albedo=0.7, vial="cylindrical", sample_time=True),
    dict(sensor="dda", sample_time=True),
    dict(sensor="dda", albedo=0.5, sample_time=True, vial="cylindrical"),
    dict(sensor="ratio", regular=True, spp=1, sample_time=True),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_paths_match_oracle(oracle, case):
    d = make(**case)
    spp = case.get("spp", 2)
    N = 16
    n = d.n_patterns * d.crop_y * d.crop_x
    rng = np.random.default_rng(0)
    pat = rng.uniform(0, 0.1, n).astype(np.float32)
    G = rng.uniform(-1, 1, (N, N, N)).astype(np.float32)
    proj = Projection(d, "cuda:0")
    out = flip_protocol(oracle, proj, d, pat, G, spp, 6, nthreads=8)
    hv = proj.count_visits(spp, 6)
    assert abs(hv - out["visits"]) <= max(2, 2e-3 * out["visits"])
    proj.close()


def test_delta_refused_without_scattering():
    d = make(sensor="delta", albedo=0.0)
    with pytest.raises(ValueError, match="purely absorptive"):
        Projection(d, "cuda:0")


def integrator_scene(method):
    """tests/test_integrators.py:7-67: 128^3 film over a d_ext cube, 100 x 128 x 128 patterns
    linspace(1, 10), collimated, distance 1.5 d_ext; glass tube (int_ior 1.514) around a
    resin tube (1.4849) with sigma_t 0.1, albedo 0.5, Rayleigh; max_depth 32, rr_depth 3,
    sample_time; the ratio sensor's majorant 10."""
    d_ext, d_int = 16.77, 15.33
    cfg = cylindrical_refraction(N=128, angles=100, size_mm=d_ext, r_int=0.5 * d_int, r_ext=0.5 * d_ext,
                                 vial_ior=1.514, medium_ior=1.4849, sigma_t=0.1, spp=128, regular_sampling=False)
    cfg["projector"]["distance"] = 1.5 * d_ext
    cfg["vial"]["height"] = 20.0
    d = desc_from_config(cfg)
    d.albedo = 0.5
    d.phase_type = _abi.PHASE_RAYLEIGH
    d.max_depth, d.rr_depth, d.sample_time, d.print_time = 32, 3, 1, 1.0
    d.sensor_type = {"dda": _abi.SENSOR_DDA, "ratio": _abi.SENSOR_RATIO, "delta": _abi.SENSOR_DELTA}[method]
    d.majorant = 10.0
    return d


def test_reverse_ad_matches_fd():
    """test_integrators.py:69-110: FD of mean(vol^2) w.r.t. a pattern scale a (dda, seed 0)
    against the reverse-mode gradient of each sensor, |rel| < 2e-4."""
    dev = "cuda:0"
    pats = torch.linspace(1, 10, 100 * 128 * 128, dtype=torch.float32, device=dev)
    a0, eps, spp = 1.0, 1e-3, 128
    proj = Projection(integrator_scene("dda"), dev)
    l1 = torch.mean(torch.square(proj.forward(pats * (a0 + eps), None, spp, 0).double()))
    l2 = torch.mean(torch.square(proj.forward(pats * (a0 - eps), None, spp, 0).double()))
    fd = float((l1 - l2) / (2 * eps))
    proj.close()
    for method in ("dda", "ratio", "delta"):
        proj = Projection(integrator_scene(method), dev)
        a = torch.tensor(a0, dtype=torch.float32, device=dev, requires_grad=True)
        vol = render(proj, a * pats, None, spp, spp, 0)
        loss = torch.mean(torch.square(vol))
        loss.backward()
        rel = abs((float(a.grad) - fd) / fd)
        print(method, float(a.grad), fd, rel)
        assert rel < 2e-4, (method, rel)
        proj.close()
