"""Where the per-ray tile kernels' lanes idle: slot / visit / cycle counters of a diagnostic build.
usage: TVAM_LIB=build_variants/libtvam_tilediag.so python tools/tile_diag.py CONFIG N ANGLES_IN_SHARD
(the library built with TVAM_CXXFLAGS=-DTVAM_TILE_DIAG=1 drtvam_amd/csrc/build.sh OUT.so).
Prints, per forward / adjoint call of the shard: the lanes' slot outcomes (marched, zero pattern,
inactive, other slice, tile-window miss), march lane utilisation (visits / (64 x the wave's
largest visit count per iteration)), and the wave cycles before the slot loop, in the per-slot
setup and in the march."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402
from drtvam_amd.configs import (cylindrical_refraction, cylindrical_scattering, desc_from_config,  # noqa: E402
                                square_occluded, square_vial)
from drtvam_amd.engine import Projection  # noqa: E402

NAMES = ["waves", "iterations", "lane_slots", "zero_pattern", "inactive", "other_slice", "window_miss",
         "marched", "visits", "wave_max_visits", "cyc_pre", "cyc_setup", "cyc_march", "tk1", "tk0", "unused"] + \
    [f"ratio_bin{b}" for b in range(8)]


def read(lib, reset=True):
    buf = (ctypes.c_ulonglong * 24)()
    assert lib.tvam_tile_diag_read(buf, 1 if reset else 0) == 0
    return dict(zip(NAMES, [int(v) for v in buf]))


def summary(d):
    slots = max(d["lane_slots"], 1)
    loop = d["tk1"] - d["tk0"]
    return {
        "slots": d["lane_slots"],
        "frac": {k: round(d[k] / slots, 4) for k in ["marched", "zero_pattern", "inactive", "other_slice", "window_miss"]},
        "visits_per_marched_lane": round(d["visits"] / max(d["marched"], 1), 2),
        "march_lane_util": round(d["visits"] / max(64 * d["wave_max_visits"], 1), 4),
        "slot_lane_util": round(d["lane_slots"] / max(64 * d["iterations"], 1), 4),
        "cycles": {"pre_loop": d["cyc_pre"], "setup": d["cyc_setup"], "march": d["cyc_march"], "loop": loop},
        "cycle_frac": {"pre_loop": round(d["cyc_pre"] / max(d["cyc_pre"] + loop, 1), 4),
                       "setup": round(d["cyc_setup"] / max(loop, 1), 4),
                       "march": round(d["cyc_march"] / max(loop, 1), 4)},
        "march_cycles_per_wave_max_visit": round(d["cyc_march"] / max(d["wave_max_visits"], 1), 2),
        "setup_cycles_per_iteration": round(d["cyc_setup"] / max(d["iterations"], 1), 1),
        "visit_ratio_hist": [round(d[f"ratio_bin{b}"] / max(d["marched"], 1), 4) for b in range(8)],
    }


def main():
    cfgname, N, na = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    if cfgname == "5":
        cfg = square_occluded(N=N, angles=N)
    elif cfgname == "5n":  # config 5 without the occluder
        cfg = square_vial(N=N, angles=N, spp=4, regular_sampling=False)
    elif cfgname == "3j":  # config 3's cylindrical vial, 4 jittered rays per pixel
        cfg = cylindrical_refraction(N=N, angles=N, spp=4, regular_sampling=False)
    else:  # "4a": config 4's first segments (albedo 0)
        cfg = cylindrical_scattering(N=N, angles=N)
        cfg["vial"]["medium"]["albedo"] = 0.0
    spp = cfg["spp"]
    a0 = N // 3
    d = desc_from_config(cfg, angle_range=(a0, a0 + na))
    d.flags |= _abi.FLAG_NO_ZERO_SKIP
    d.active_total = N * N * N
    n = na * N * N
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(n, generator=g) * 0.1).cuda()
    G = (torch.rand((N, N, N), generator=g) * 2 - 1).cuda()
    lib = _abi.load_library()
    lib.tvam_tile_diag_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    p = Projection(d, "cuda:0")
    torch.cuda.synchronize()
    read(lib)
    p.forward(x, None, spp, 1)
    torch.cuda.synchronize()
    fwd = read(lib)
    p.adjoint(G, n, None, spp, 2)
    torch.cuda.synchronize()
    adj = read(lib)
    out = {"config": cfgname, "n": N, "angles": na, "forward": {"raw": fwd, **summary(fwd)},
           "adjoint": {"raw": adj, **summary(adj)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
