"""DMD projectors (mirror of drtvam/projector.py).

``active_data`` (float32, one value per active DMD pixel and angle) and
``active_pixels`` (flat index ``angle*H*W + row*W + col``) keep the reference's
meaning and order (projector.py:60-99).  They live in torch tensors on the
engine's device.  ``dense`` is True while ``active_pixels`` is exactly the
dense crop enumeration of projector.py:90-98, in which case the kernels index
``active_data`` directly and ``active_pixels`` is never read.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .motion import Motion, motions
from . import _abi


def default_device() -> torch.device:
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def load_patterns(filepath):
    """.npy / .npz pattern stacks or a directory of EXR images (projector.py:8-39)."""
    if os.path.isfile(filepath):
        if filepath.endswith(".npy"):
            patterns = np.load(filepath)
        elif filepath.endswith(".npz"):
            patterns = np.load(filepath)
            if len(patterns.files) != 1:
                raise ValueError(f"Expected a single array in the npz file, but got {len(patterns.files)} arrays.")
            patterns = patterns[patterns.files[0]]
        else:
            raise ValueError(f"Unsupported file format for patterns: {os.path.splitext(filepath)[1]}")
        if len(patterns.shape) != 3:
            raise ValueError(f"Patterns must be 3D, but got a tensor of shape {patterns.shape}.")
        return np.ascontiguousarray(patterns, dtype=np.float32)
    import glob
    from .exr import read_exr
    filenames = glob.glob(os.path.join(filepath, "*.exr"))
    if len(filenames) == 0:
        raise ValueError("No patterns found in the specified directory. Please make sure the patterns are in EXR format.")
    imgs = None
    for i, fn in enumerate(sorted(filenames)):
        img = read_exr(fn)
        if i == 0:
            h, w, _ = img.shape
            imgs = np.empty((len(filenames), h, w), dtype=np.float32)
        elif img.shape[:2] != (h, w):
            raise ValueError(f"File '{fn}' has a different resolution ({img.shape[0]}x{img.shape[1]}) than the previous "
                             f"files ({h}x{w}). All patterns are expected to have the same resolution.")
        # mi.TensorXf(Bitmap).array scattered over h*w entries: the first h*w values of the
        # interleaved [h, w, c] image (projector.py:34-35)
        imgs[i] = img.reshape(-1)[:h * w].reshape(h, w)
    return imgs


class TVAMProjector:
    def __init__(self, props):
        self.device = torch.device(props.get('device', default_device()))
        self.m_sampler = props.get('sampler', {'type': 'independent'})

        if 'patterns' in props:
            p = props['patterns']
            if isinstance(p, str):
                patterns = load_patterns(p)
            elif isinstance(p, torch.Tensor):
                patterns = p.detach().to(torch.float32).cpu().numpy()
            elif isinstance(p, np.ndarray):
                patterns = np.asarray(p, dtype=np.float32)
            else:
                raise ValueError(f"[{self.__class__.__name__}] patterns must be of type TensorXf")
            if len(patterns.shape) != 3:
                raise ValueError(f"[{self.__class__.__name__}] Patterns must be 3D, but got a tensor of shape {patterns.shape}.")
            n, h, w = patterns.shape
            self.n_patterns = n
            self.res = (w, h)
            self.crop = self.res
            self.crop_offset = (0, 0)
            flat = torch.from_numpy(np.ascontiguousarray(patterns).reshape(-1))
            if props.get('filter_nonzero', False):
                idx = torch.nonzero(flat > 0).reshape(-1).to(torch.int32)
                self.active_pixels = idx.to(self.device)
                self.active_data = flat[idx.long()].to(self.device)
                self.dense = False
            else:
                self.active_data = flat.to(self.device)
                self.active_pixels = torch.arange(n * h * w, dtype=torch.int32, device=self.device)
                self.dense = True
        else:
            self.n_patterns = props.get('n_patterns', 1000)
            resx = props.get('resx', 256)
            resy = props.get('resy', 256)
            self.res = (resx, resy)
            cropx = props.get('cropx', resx)
            cropy = props.get('cropy', resy)
            self.crop = (cropx, cropy)
            if cropx > resx or cropy > resy:
                raise ValueError(f"[{self.__class__.__name__}] Crop resolution ({self.crop}) must be smaller than the base resolution ({self.res}).")
            self.crop_offset = (props.get('crop_offset_x', 0), props.get('crop_offset_y', 0))
            if self.crop_offset[0] + cropx > resx or self.crop_offset[1] + cropy > resy:
                raise ValueError(f"[{self.__class__.__name__}] With the specified crop offset ({self.crop_offset}), the cropped region ({self.crop}) extends beyond the base resolution ({self.res}).")
            n_crop = cropx * cropy
            self.active_data = torch.zeros(self.n_patterns * n_crop, dtype=torch.float32, device=self.device)
            self.active_pixels = self.dense_pixels().to(self.device)
            self.dense = True

        if "motion" not in props:
            raise ValueError(f"[{self.__class__.__name__}] Missing field 'motion'.")
        if isinstance(props['motion'], Motion):
            self.motion = props['motion']
        elif isinstance(props['motion'], str):
            if props['motion'] not in motions.keys():
                raise ValueError(f"[{self.__class__.__name__}] Invalid motion type: {props['motion']}")
            self.motion = motions[props['motion']](props)
        else:
            raise ValueError(f"[{self.__class__.__name__}] motion must be either a dict or a Motion instance")

    # --- reference API ---------------------------------------------------
    def sampler(self):
        return self.m_sampler

    def active_size(self):
        return int(self.active_data.numel())

    def size(self):
        return (self.n_patterns, self.res[1], self.res[0])

    def dense_pixels(self) -> torch.Tensor:
        """active_pixels of the full crop, in the order of projector.py:92-98."""
        cropx, cropy = self.crop
        ox, oy = self.crop_offset
        resx, resy = self.res
        crop_idx = torch.arange(cropx * cropy, dtype=torch.int64)
        pix = (oy + crop_idx // cropx) * resx + crop_idx % cropx + ox
        a = torch.arange(self.n_patterns, dtype=torch.int64).repeat_interleave(cropx * cropy)
        return (a * (resx * resy) + pix.repeat(self.n_patterns)).to(torch.int32)

    def patterns(self) -> torch.Tensor:
        """Full pattern stack [n, H, W] (projector.py:125-129)."""
        out = torch.zeros(self.n_patterns * self.res[0] * self.res[1], dtype=torch.float32, device=self.device)
        out[self.active_pixels.long()] = self.active_data.detach().to(out.device)
        return out.reshape(self.n_patterns, self.res[1], self.res[0])

    def set_active(self, active_data: torch.Tensor, active_pixels: torch.Tensor | None = None):
        """params.update() equivalent (projector.py:131-139)."""
        if active_pixels is not None:
            self.active_pixels = active_pixels.to(device=self.device, dtype=torch.int32).contiguous()
            dp = self.dense_pixels().to(self.device)
            self.dense = bool(dp.numel() == self.active_pixels.numel() and torch.equal(dp, self.active_pixels))
        self.active_data = active_data
        if self.active_data.numel() != self.active_pixels.numel():
            raise ValueError(f"[{self.__class__.__name__}] active_data and active_pixels must have the same length.")

    def fill_desc(self, desc: _abi.TvamDesc) -> None:
        raise NotImplementedError

    def _fill_common(self, desc):
        from .motion import CircularMotion
        if not isinstance(self.motion, CircularMotion):
            raise NotImplementedError("only circular motion is supported by the GPU engine")
        desc.n_patterns = int(self.n_patterns)
        desc.res_x, desc.res_y = int(self.res[0]), int(self.res[1])
        desc.crop_x, desc.crop_y = int(self.crop[0]), int(self.crop[1])
        desc.crop_offset_x, desc.crop_offset_y = int(self.crop_offset[0]), int(self.crop_offset[1])
        desc.distance = float(self.motion.distance)
        desc.clockwise = int(bool(self.motion.clockwise))


class CollimatedProjector(TVAMProjector):
    """Orthographic DMD: parallel rays along the projector axis (projector.py:167-196)."""

    def __init__(self, props):
        super().__init__(props)
        ps = props['pixel_size']
        if isinstance(ps, (int, float)):
            self.pixel_size = (float(ps), float(ps))
        elif isinstance(ps, (tuple, list)) and len(ps) == 2:
            self.pixel_size = (float(ps[0]), float(ps[1]))
        else:
            raise ValueError(f"[{self.__class__.__name__}] pixel_size must be a float or a Point2f")
        self.emitter_size = (self.res[0] * self.pixel_size[0], self.res[1] * self.pixel_size[1])

    def fill_desc(self, desc):
        self._fill_common(desc)
        desc.projector_type = _abi.PROJECTOR_COLLIMATED
        desc.pixel_size_x, desc.pixel_size_y = self.pixel_size

    def to_string(self):
        return ('CollimatedProjector[\n'
                f'    pattern count = {self.n_patterns},\n'
                f'    pattern resolution = {self.res},\n'
                f'    emitter_size = {self.emitter_size},\n'
                ']')


class TelecentricProjector(TVAMProjector):
    """Telecentric lens projector (projector.py:199-237); not on the GPU path yet."""

    def __init__(self, props):
        super().__init__(props)
        self.pixel_size = props['pixel_size']
        self.aperture_radius = props['aperture_radius']
        self.focus_distance = props['focus_distance']


class LensProjector(TVAMProjector):
    """Perspective lens projector (projector.py:241-296); not on the GPU path yet."""

    def __init__(self, props):
        super().__init__(props)
        self.aperture_radius = props['aperture_radius']
        self.focus_distance = props['focus_distance']


emitters = {
    'collimated': CollimatedProjector,
    'lens': LensProjector,
    'telecentric': TelecentricProjector,
}
