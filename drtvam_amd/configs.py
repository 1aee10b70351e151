"""Workload configurations of BASELINE.json, as drtvam JSON-style config dicts.

config 1 / 2: index-matched "Benchy" scene (README.md:118-123: 10 mm print,
25 um pixels at N=400), N^3 voxels, N angles, N x N DMD, 1 ray/pixel,
regular sampling.  benchy.ply is not in the reference
snapshot (.MISSING_LARGE_BLOBS), so the target is analytic; the target only
enters the loss, never the projection.
"""
from __future__ import annotations

import copy

from . import _abi


def benchy_index_matched(N: int = 400, angles: int | None = None, size_mm: float = 10.0, r: float = 8.0,
                         sigma_t: float = 0.03, spp: int = 1, regular_sampling: bool = True, n_steps: int = 40):
    A = N if angles is None else angles
    pix = size_mm / N
    return {
        "vial": {"type": "index_matched", "r": r, "height": 40.0,
                 "medium": {"ior": 1.0, "extinction": sigma_t, "albedo": 0.0}},
        "projector": {"type": "collimated", "n_patterns": A, "resx": N, "resy": N, "pixel_size": pix,
                      "motion": "circular", "distance": 20.0},
        "sensor": {"type": "dda", "scalex": size_mm, "scaley": size_mm, "scalez": size_mm,
                   "film": {"type": "vfilm", "resx": N, "resy": N, "resz": N}},
        "target": {"analytic": "box_hole"},
        "loss": {"type": "threshold", "tl": 0.9, "tu": 0.95},
        "spp": spp,
        "regular_sampling": regular_sampling,
        "n_steps": n_steps,
        "time": 1.0,
    }


def cylindrical_refraction(N: int = 400, angles: int | None = None, size_mm: float = 10.0, r_int: float = 8.0,
                           r_ext: float = 9.0, vial_ior: float = 1.54, medium_ior: float = 1.40,
                           sigma_t: float = 0.03, spp: int = 1, regular_sampling: bool = True, n_steps: int = 40):
    """Config 3 (BASELINE.json): the config 2 scene in a glass tube (r_int / r_ext, dielectric
    interfaces air|glass|resin; IORs of tests/files/box_hole_cylindrical.json), no scattering."""
    cfg = benchy_index_matched(N=N, angles=angles, size_mm=size_mm, sigma_t=sigma_t, spp=spp,
                               regular_sampling=regular_sampling, n_steps=n_steps)
    cfg["vial"] = {"type": "cylindrical", "r_int": r_int, "r_ext": r_ext, "ior": vial_ior, "height": 40.0,
                   "medium": {"ior": medium_ior, "extinction": sigma_t, "albedo": 0.0}}
    return cfg


def cylindrical_scattering(N: int = 400, angles: int | None = None, spp: int = 16, sigma_t: float = 0.1,
                           albedo: float = 0.5, phase: str = "rayleigh", n_steps: int = 40):
    """Config 4 (BASELINE.json): the config 3 tube around a scattering resin (the medium of
    tests/files/box_hole_cylindrical.json: extinction 0.1 / mm, albedo 0.5, Rayleigh phase),
    16 jittered rays per pixel."""
    cfg = cylindrical_refraction(N=N, angles=angles, sigma_t=sigma_t, spp=spp, regular_sampling=False,
                                 n_steps=n_steps)
    cfg["vial"]["medium"]["albedo"] = albedo
    cfg["vial"]["medium"]["phase"] = {"type": phase}
    return cfg


def square_vial(N: int = 400, angles: int | None = None, size_mm: float = 5.0, w_int: float = 7.191,
                w_ext: float = 7.6, vial_ior: float = 1.3, medium_ior: float = 1.15, sigma_t: float = 0.06,
                spp: int = 1, regular_sampling: bool = True, occluders=(), n_steps: int = 40):
    """A square glass vial (the vial and resin of tests/files/box_hole_occlusion.json: w_int 7.191,
    w_ext 7.6, glass ior 1.3, resin ior 1.15, extinction 0.06 / mm), optional occluder PLY meshes."""
    cfg = benchy_index_matched(N=N, angles=angles, size_mm=size_mm, sigma_t=sigma_t, spp=spp,
                               regular_sampling=regular_sampling, n_steps=n_steps)
    cfg["vial"] = {"type": "square", "w_int": w_int, "w_ext": w_ext, "ior": vial_ior,
                   "medium": {"ior": medium_ior, "extinction": sigma_t, "albedo": 0.0},
                   "occlusions": [{"filename": f} for f in occluders]}
    return cfg


def square_occluded(N: int = 800, angles: int | None = None, spp: int = 4, occluder: str | None = None,
                    n_steps: int = 40):
    """Config 5 (BASELINE.json): overprinting around an occluder in a square vial -- the scene of
    tests/files/box_hole_occlusion.json (5 mm film, square vial, the 2 x 1 x 0.5 mm occluder box
    of tests/files/occlusion.ply) at N^3 voxels, N angles, N x N DMD, 4 jittered rays per pixel."""
    import os
    occ = occluder or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                   "occlusion.ply")
    return square_vial(N=N, angles=angles, spp=spp, regular_sampling=False, occluders=(occ,), n_steps=n_steps)


# tests/files/box_hole_square.json, box_hole_occlusion.json and box_hole_scattering.json of
# the reference (data, restated; the occluder / target paths are set by the caller)
BOX_HOLE_SQUARE = {
    "vial": {"type": "square", "w_int": 10.191, "w_ext": 12.408, "ior": 1.54,
             "medium": {"ior": 1.347, "phase": {"type": "rayleigh"}, "extinction": 0.03, "albedo": 0.0}},
    "projector": {"type": "collimated", "n_patterns": 200, "resx": 200, "resy": 20, "pixel_size": 50e-3,
                  "motion": "circular", "distance": 20},
    "sensor": {"type": "dda", "scalex": 5, "scaley": 5, "scalez": 1.25,
               "film": {"type": "vfilm", "resx": 100, "resy": 100, "resz": 50}},
    "target": {"filename": "tests/files/box_hole.ply", "size": 4.0},
    "loss": {"type": "threshold", "tl": 0.85, "tu": 0.95},
    "progressive": True,
    "n_steps": 30,
}
BOX_HOLE_OCCLUSION = {
    "vial": {"type": "square", "w_int": 7.191, "w_ext": 7.6, "ior": 1.3,
             "medium": {"ior": 1.15, "phase": {"type": "rayleigh"}, "extinction": 0.06, "albedo": 0.0},
             "occlusions": [{"filename": "tests/files/occlusion.ply"}]},
    "projector": BOX_HOLE_SQUARE["projector"],
    "sensor": BOX_HOLE_SQUARE["sensor"],
    "target": {"filename": "tests/files/box_hole.ply", "size": 4.0},
    "loss": {"type": "threshold", "tl": 0.9, "tu": 0.97},
    "progressive": True,
    "n_steps": 30,
}
BOX_HOLE_SCATTERING = {
    "vial": {"type": "square", "w_int": 7.0, "w_ext": 8.0, "ior": 1.24,
             "medium": {"ior": 1.347, "phase": {"type": "rayleigh"}, "extinction": 0.09, "albedo": 0.9}},
    "projector": BOX_HOLE_SQUARE["projector"],
    "sensor": BOX_HOLE_SQUARE["sensor"],
    "target": {"filename": "tests/files/box_hole.ply", "size": 4.0},
    "loss": {"type": "threshold", "tl": 0.35, "tu": 0.55},
    "filter_radon": True,
    "spp_ref": 16,
    "spp": 4,
    "spp_grad": 16,
    "progressive": True,
    "n_steps": 30,
}

# tests/files/box_hole_square_different_thresholds.json: the square vial of box_hole_scattering.json
# (w_int 7 / w_ext 8, ior 1.24, extinction 0.09) with a non-scattering resin and thresholds 0.35 / 0.55
BOX_HOLE_SQUARE_DIFFERENT_THRESHOLDS = {
    "vial": {"type": "square", "w_int": 7.0, "w_ext": 8.0, "ior": 1.24,
             "medium": {"ior": 1.347, "phase": {"type": "rayleigh"}, "extinction": 0.09, "albedo": 0.0}},
    "projector": BOX_HOLE_SQUARE["projector"],
    "sensor": BOX_HOLE_SQUARE["sensor"],
    "target": {"filename": "tests/files/box_hole.ply", "size": 4.0},
    "loss": {"type": "threshold", "tl": 0.35, "tu": 0.55},
    "progressive": True,
    "n_steps": 30,
}

# tests/files/box_hole_index_matched.json of the reference (data, restated)
BOX_HOLE_INDEX_MATCHED = {
    "vial": {"type": "index_matched", "r": 2.9,
             "medium": {"ior": 1.347, "phase": {"type": "rayleigh"}, "extinction": 0.03, "albedo": 0.0}},
    "projector": {"type": "collimated", "n_patterns": 200, "resx": 200, "resy": 20, "pixel_size": 50e-3,
                  "motion": "circular", "distance": 20},
    "sensor": {"type": "dda", "scalex": 5, "scaley": 5, "scalez": 1.25,
               "film": {"type": "vfilm", "resx": 100, "resy": 100, "resz": 50}},
    "target": {"filename": "tests/files/box_hole.ply", "size": 4.0},
    "loss": {"type": "threshold", "tl": 0.85, "tu": 0.95},
    "progressive": True,
    "n_steps": 30,
}

# tests/files/box_hole_cylindrical.json of the reference (data, restated): glass tube
# r_int 7 / r_ext 8 (ior 1.54) around a scattering resin (ior 1.40, albedo 0.5)
BOX_HOLE_CYLINDRICAL = {
    "vial": {"type": "cylindrical", "r_int": 7, "r_ext": 8, "ior": 1.54,
             "medium": {"ior": 1.40, "phase": {"type": "rayleigh"}, "extinction": 0.1, "albedo": 0.5}},
    "projector": {"type": "collimated", "n_patterns": 200, "resx": 200, "resy": 20, "pixel_size": 50e-3,
                  "motion": "circular", "distance": 20},
    "sensor": {"type": "dda", "scalex": 5, "scaley": 5, "scalez": 1.25,
               "film": {"type": "vfilm", "resx": 100, "resy": 100, "resz": 50}},
    "target": {"filename": "tests/files/box_hole.ply", "size": 4.0,
               "box_center_x": 0, "box_center_y": 0, "box_center_z": 0},
    "loss": {"type": "threshold", "tl": 0.85, "tu": 0.95},
    "progressive": True,
    "n_steps": 30,
}


def desc_from_config(config, angle_range=None, tile: int = 0) -> _abi.TvamDesc:
    """tvam_desc of a config through the plugin classes (no GPU needed)."""
    from .optimize import load_scene
    from .scene import load_dict
    from .integrators import VolumeIntegrator

    cfg = copy.deepcopy(config)
    cfg["projector"]["device"] = "cpu"
    if "filename" in cfg.get("target", {}):
        cfg["target"] = {"analytic": "box_hole"}
    scene = load_dict(load_scene(cfg))
    integ = VolumeIntegrator({
        "max_depth": cfg.get("max_depth", 6), "rr_depth": cfg.get("rr_depth", 6), "print_time": cfg.get("time", 1.0),
        "transmission_only": cfg.get("transmission_only", True),
        "regular_sampling": cfg.get("regular_sampling", False), "angle_range": angle_range, "tile": tile})
    return integ.desc(scene, scene.sensor_by_id("sensor"))
