"""Printing-medium containers (mirror of drtvam/geometry.py).

Each container keeps the reference's constructor properties and validation.
Instead of emitting a Mitsuba scene dictionary, ``to_dict()`` returns the
same keys with our own shape dictionaries and ``fill_desc()`` writes the
container into the C descriptor consumed by libtvam.so.
"""
from __future__ import annotations

from . import _abi


class Container:
    """Base class: medium IOR, extinction, albedo, phase function, occlusions (geometry.py:4-72)."""

    def __init__(self, params):
        if 'medium' not in params.keys():
            raise ValueError(f"[{self.__class__.__name__}] Missing field 'medium'.")
        medium = params['medium']
        self.medium_ior = medium['ior']
        self.sigma_t = medium['extinction']
        self.albedo = medium['albedo']
        self.occlusions = params.get('occlusions', [])

        if 'phase' in medium.keys():
            self.medium_phase = medium['phase']
        elif self.albedo > 0.:
            raise ValueError(f"[{self.__class__.__name__}] Tried to load a scattering medium without specifying a phase function.")
        else:
            self.medium_phase = None

    def medium_dict(self):
        medium_dict = {
            'type': 'homogeneous',
            'sigma_t': self.sigma_t,
            'albedo': self.albedo,
        }
        if self.medium_phase is not None:
            medium_dict['phase'] = self.medium_phase
        return medium_dict

    def to_dict(self):
        raise NotImplementedError

    def fill_desc(self, desc: _abi.TvamDesc) -> None:
        raise NotImplementedError(f"{self.__class__.__name__} is not supported by the GPU engine yet")

    def _fill_medium(self, desc):
        desc.sigma_t = float(self.sigma_t)
        desc.albedo = float(self.albedo)
        phase = self.medium_phase or {"type": "isotropic"}  # Mitsuba's default phase function
        kinds = {"isotropic": _abi.PHASE_ISOTROPIC, "rayleigh": _abi.PHASE_RAYLEIGH, "hg": _abi.PHASE_HG}
        if phase.get("type") not in kinds:
            raise NotImplementedError(f"phase function '{phase.get('type')}' is not supported by the GPU engine")
        desc.phase_type = kinds[phase["type"]]
        desc.phase_g = float(phase.get("g", 0.8))  # Mitsuba hg default g
        desc.medium_ior = lookup_ior(self.medium_ior)
        if self.occlusions:
            import numpy as np
            from .utils import read_ply
            tris = []
            for occ in self.occlusions:
                bsdf = occ.get("bsdf")
                if bsdf is not None and not (bsdf.get("type") == "diffuse" and
                                             float(bsdf.get("reflectance", {}).get("value", 0.0)) == 0.0):
                    raise NotImplementedError("occluders must be black diffuse (the reference default)")
                v, f = read_ply(occ["filename"])
                tris.append(np.asarray(v, np.float32)[np.asarray(f)])
            desc.set_occluders(np.concatenate(tris))


# Named refractive indices (Mitsuba's ior table, restated for the names a config may use)
IOR_TABLE = {
    'vacuum': 1.0, 'helium': 1.000036, 'hydrogen': 1.000132, 'air': 1.000277, 'carbon dioxide': 1.00045,
    'water': 1.3330, 'acetone': 1.36, 'ethanol': 1.361, 'carbon tetrachloride': 1.461, 'glycerol': 1.4729,
    'benzene': 1.501, 'silicone oil': 1.52045, 'bromine': 1.661, 'water ice': 1.31, 'fused quartz': 1.458,
    'pyrex': 1.470, 'acrylic glass': 1.49, 'polypropylene': 1.49, 'bk7': 1.5046, 'sodium chloride': 1.544,
    'amber': 1.55, 'pet': 1.5750, 'diamond': 2.419,
}


def lookup_ior(v) -> float:
    if isinstance(v, str):
        if v not in IOR_TABLE:
            raise ValueError(f"Unknown IOR name '{v}'")
        return float(IOR_TABLE[v])
    return float(v)


class IndexMatchedVial(Container):
    """Null-BSDF open cylinder of radius r around the z axis (geometry.py:75-96)."""

    def __init__(self, params):
        super().__init__(params)
        self.r = params['r']
        self.height = params.get('height', 40.)

    def to_dict(self):
        return {
            'printing_medium': self.medium_dict(),
            'vial_exterior': {
                'type': 'cylinder',
                'p0': [0., 0., -0.5 * self.height],
                'p1': [0., 0., 0.5 * self.height],
                'radius': self.r,
                'bsdf': {'type': 'null'},
                'interior': {'type': 'ref', 'id': 'printing_medium'},
            },
        }

    def fill_desc(self, desc):
        self._fill_medium(desc)
        desc.vial_type = _abi.VIAL_INDEX_MATCHED
        desc.vial_r = float(self.r)
        desc.vial_height = float(self.height)


class CylindricalVial(Container):
    """Glass cylinder r_ext / r_int with dielectric interfaces (geometry.py:142-183)."""

    def __init__(self, params):
        super().__init__(params)
        self.r_int = params['r_int']
        self.r_ext = params['r_ext']
        self.height = params.get('height', 40.)
        self.vial_ior = params['ior']

    def to_dict(self):
        return {
            'printing_medium': self.medium_dict(),
            'vial_exterior': {'type': 'cylinder', 'p0': [0., 0., -0.5 * self.height], 'p1': [0., 0., 0.5 * self.height],
                              'radius': self.r_ext,
                              'bsdf': {'type': 'dielectric', 'int_ior': self.vial_ior, 'ext_ior': 'air'}},
            'vial_interior': {'type': 'cylinder', 'p0': [0., 0., -0.5 * self.height], 'p1': [0., 0., 0.5 * self.height],
                              'radius': self.r_int,
                              'bsdf': {'type': 'dielectric', 'ext_ior': self.vial_ior, 'int_ior': self.medium_ior},
                              'interior': {'type': 'ref', 'id': 'printing_medium'}},
        }

    def fill_desc(self, desc):
        self._fill_medium(desc)
        desc.vial_type = _abi.VIAL_CYLINDRICAL
        desc.vial_r = float(self.r_int)
        desc.vial_r_ext = float(self.r_ext)
        desc.vial_height = float(self.height)
        desc.vial_ior = lookup_ior(self.vial_ior)


class SquareVial(Container):
    """Glass cuboid w_ext / w_int (geometry.py:186-219)."""

    def __init__(self, params):
        super().__init__(params)
        self.w_int = params['w_int']
        self.w_ext = params['w_ext']
        self.height = params.get('height', 100.)
        self.vial_ior = params['ior']

    def fill_desc(self, desc):
        self._fill_medium(desc)
        desc.vial_type = _abi.VIAL_SQUARE
        desc.vial_r = 0.5 * float(self.w_int)
        desc.vial_r_ext = 0.5 * float(self.w_ext)
        desc.vial_height = float(self.height)
        desc.vial_ior = lookup_ior(self.vial_ior)

    def to_dict(self):
        return {'printing_medium': self.medium_dict(),
                'vial_exterior': {'type': 'cube', 'scale': (0.5 * self.w_ext, 0.5 * self.w_ext, 0.5 * self.height),
                                  'bsdf': {'type': 'dielectric', 'int_ior': self.vial_ior}},
                'vial_interior': {'type': 'cube', 'scale': (0.5 * self.w_int, 0.5 * self.w_int, 0.45 * self.height),
                                  'bsdf': {'type': 'dielectric', 'ext_ior': self.vial_ior, 'int_ior': self.medium_ior},
                                  'interior': {'type': 'ref', 'id': 'printing_medium'}}}


class CustomVial(Container):
    """PLY inner/outer vial meshes (geometry.py:98-138)."""

    def __init__(self, params):
        super().__init__(params)
        if "filename_vial_outer" not in params.keys() or "filename_vial_inner" not in params.keys():
            raise ValueError(f"[{self.__class__.__name__}] Missing fields 'filename_vial_outer' or 'filename_vial_inner' for custom vial.")
        self.vial_ior = params['ior']
        self.filename_vial_outer = params["filename_vial_outer"]
        self.filename_vial_inner = params["filename_vial_inner"]

    def to_dict(self):
        return {'printing_medium': self.medium_dict(),
                'vial_exterior': {'type': 'ply', 'filename': self.filename_vial_outer},
                'vial_interior': {'type': 'ply', 'filename': self.filename_vial_inner}}


class DoubleCylindricalVial(Container):
    """Two nested glass cylinders (geometry.py:222-308)."""

    def __init__(self, params):
        super().__init__(params)
        self.r_ext_outer = params['r_ext_outer']
        self.r_int_outer = params['r_int_outer']
        self.r_ext_inner = params['r_ext_inner']
        self.r_int_inner = params['r_int_inner']
        self.height = params.get('height', 40.)
        self.vial_ior_inner = params['ior_inner']
        self.vial_ior_outer = params['ior_outer']
        self.inside_inner_ior = params['ior_inside_inner']

    def to_dict(self):
        return {'printing_medium': self.medium_dict()}


geometries = {
    'index_matched': IndexMatchedVial,
    'cylindrical': CylindricalVial,
    'square': SquareVial,
    'custom': CustomVial,
    'double_cylindrical': DoubleCylindricalVial,
}
