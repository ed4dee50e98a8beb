"""BMP images of field slices (reference ``BMPDumper.cpp``, ``BMPHelper.cpp``,
``BMPLoader.cpp``) without EasyBMP: 24-bit uncompressed BMP written and read
with numpy.

* Palette ``rgb`` (reference blue-green-red, ``BMPHelper.cpp:61-95``): values
  normalised to the region's ``[min, max]``; lower half blue->green, upper
  half green->red.  ``gray``: linear grey (``BMPHelper.cpp:101-115``).
* 1D grids: an ``N x 1`` image; 2D: ``Nx x Ny`` (pixel ``(i, j)``); 3D: one image
  per slice along the orthogonal axis (default z), named
  ``<file><slice>-Re.bmp`` (``BMPDumper.cpp:1166``).  Complex fields also get
  ``-Im`` and ``-Mod`` images.
* The loader inverts the palette given the ``[min, max]`` used for writing
  (the reference's BMPLoader takes them from settings and has no 3D support;
  here 3D slice stacks load too).
"""

from __future__ import annotations

import os
import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .naming import GridFileType, grid_file_name, levels


def palette_rgb(v: np.ndarray, vmin: float, vmax: float) -> np.ndarray:
    """float array -> (..., 3) uint8 RGB, reference blue-green-red scheme."""
    rng = vmax - vmin
    value = v.astype(np.float64) - vmin
    half = rng / 2.0
    out = np.zeros(v.shape + (3,), dtype=np.uint8)
    if rng == 0:
        out[..., 2] = 255  # tmp = 0 -> pure blue
        return out
    hi = value > half
    tmp_hi = np.where(hi, (value - half) / half, 0.0)
    tmp_lo = np.where(hi, 0.0, value / half)
    r = np.where(hi, tmp_hi * 255, 0.0)
    g = np.where(hi, (1.0 - tmp_hi) * 255, tmp_lo * 255)
    b = np.where(hi, 0.0, (1.0 - tmp_lo) * 255)
    out[..., 0] = np.clip(r, 0, 255).astype(np.uint8)
    out[..., 1] = np.clip(g, 0, 255).astype(np.uint8)
    out[..., 2] = np.clip(b, 0, 255).astype(np.uint8)
    return out


def palette_gray(v: np.ndarray, vmin: float, vmax: float) -> np.ndarray:
    rng = vmax - vmin
    g = np.zeros(v.shape) if rng == 0 else (v.astype(np.float64) - vmin) / rng * 255
    g = np.clip(g, 0, 255).astype(np.uint8)
    return np.stack([g, g, g], axis=-1)


def inverse_rgb(px: np.ndarray, vmin: float, vmax: float) -> np.ndarray:
    """(..., 3) uint8 -> float values (inverse of :func:`palette_rgb`, up to
    8-bit quantisation)."""
    rng = vmax - vmin
    half = rng / 2.0
    r = px[..., 0].astype(np.float64)
    g = px[..., 1].astype(np.float64)
    b = px[..., 2].astype(np.float64)
    upper = (b == 0) & (r > 0)
    val = np.where(upper, half + r / 255.0 * half, g / 255.0 * half)
    return val + vmin


def inverse_gray(px: np.ndarray, vmin: float, vmax: float) -> np.ndarray:
    return px[..., 0].astype(np.float64) / 255.0 * (vmax - vmin) + vmin


def write_bmp(path: str, rgb: np.ndarray) -> None:
    """rgb: (width, height, 3) with pixel (x, y), y = 0 the top row."""
    w, h = rgb.shape[0], rgb.shape[1]
    row_bytes = (w * 3 + 3) & ~3
    img = np.zeros((h, row_bytes), dtype=np.uint8)
    # BMP rows are bottom-up, pixels stored BGR
    bgr = rgb[:, :, ::-1].transpose(1, 0, 2)  # (h, w, 3), row y
    img[:, : w * 3] = bgr[::-1].reshape(h, w * 3)
    size = 54 + img.size
    header = struct.pack("<2sIHHI", b"BM", size, 0, 0, 54)
    info = struct.pack("<IiiHHIIiiII", 40, w, h, 1, 24, 0, img.size, 2835, 2835, 0, 0)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(header)
        f.write(info)
        f.write(img.tobytes())


def read_bmp(path: str) -> np.ndarray:
    """-> (width, height, 3) RGB uint8 with y = 0 the top row."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:2] != b"BM":
        raise ValueError("%s is not a BMP" % path)
    off = struct.unpack_from("<I", data, 10)[0]
    w, h = struct.unpack_from("<ii", data, 18)
    bpp = struct.unpack_from("<H", data, 28)[0]
    if bpp != 24:
        raise ValueError("only 24-bit BMP is supported")
    top_down = h < 0
    h = abs(h)
    row_bytes = (w * 3 + 3) & ~3
    img = np.frombuffer(data, dtype=np.uint8, count=row_bytes * h, offset=off).reshape(h, row_bytes)
    img = img[:, : w * 3].reshape(h, w, 3)
    if not top_down:
        img = img[::-1]
    return img[:, :, ::-1].transpose(1, 0, 2).copy()


def _slices(a: np.ndarray, axis: int):
    for s in range(a.shape[axis]):
        yield s, np.take(a, s, axis=axis)


class BMPDumper:
    def __init__(self, step=0, kind=GridFileType.CURRENT, rank=0, name="", directory=".", palette="rgb",
                 orth_axis=2):
        self.step, self.kind, self.rank, self.name = step, kind, rank, name
        self.directory, self.palette, self.orth_axis = directory, palette, orth_axis

    def init(self, step, kind, rank, name):
        self.step, self.kind, self.rank, self.name = step, kind, rank, name

    def _img(self, a: np.ndarray, vmin, vmax):
        return palette_rgb(a, vmin, vmax) if self.palette == "rgb" else palette_gray(a, vmin, vmax)

    def dump_grid(self, t: torch.Tensor, imag: Optional[torch.Tensor] = None, start=None, end=None,
                  dim: Optional[int] = None) -> List[str]:
        """Write images of ``t[start:end]``; returns the file names."""
        a = t.detach().cpu().double().numpy()
        if start is not None:
            sl = tuple(slice(start[d], end[d]) for d in range(a.ndim))
            a = a[sl]
        parts = [("Re", a)]
        if imag is not None:
            b = imag.detach().cpu().double().numpy()
            if start is not None:
                b = b[sl]
            parts += [("Im", b), ("Mod", np.sqrt(a * a + b * b))]
        dim = dim if dim is not None else sum(1 for s in a.shape if s > 1) or 1
        files = []
        for lv in levels(self.kind):
            base = grid_file_name(self.step, lv, self.rank, self.name, self.directory)
            for tag, arr in parts:
                vmin, vmax = float(arr.min()), float(arr.max())
                if dim == 3:
                    s0 = start[self.orth_axis] if start is not None else 0
                    for s, sl2 in _slices(arr, self.orth_axis):
                        p = "%s%d-%s.bmp" % (base, s + s0, tag)
                        write_bmp(p, self._img(sl2, vmin, vmax))
                        files.append(p)
                else:
                    a2 = arr.reshape(arr.shape[0], -1) if arr.ndim > 1 else arr.reshape(-1, 1)
                    if dim == 2 and arr.ndim == 3:
                        a2 = arr[:, :, 0] if arr.shape[2] == 1 else arr.reshape(arr.shape[0], -1)
                    p = "%s-%s.bmp" % (base, tag)
                    write_bmp(p, self._img(a2, vmin, vmax))
                    files.append(p)
        return files


class BMPLoader:
    def __init__(self, step=0, kind=GridFileType.CURRENT, rank=0, name="", directory=".", palette="rgb",
                 orth_axis=2):
        self.step, self.kind, self.rank, self.name = step, kind, rank, name
        self.directory, self.palette, self.orth_axis = directory, palette, orth_axis

    def load_grid(self, shape: Sequence[int], vmin: float, vmax: float,
                  level: GridFileType = GridFileType.CURRENT, tag: str = "Re") -> torch.Tensor:
        base = grid_file_name(self.step, level, self.rank, self.name, self.directory)
        inv = inverse_rgb if self.palette == "rgb" else inverse_gray
        shape = tuple(shape)
        dim = sum(1 for s in shape if s > 1) or 1
        if dim == 3:
            out = np.zeros(shape)
            for s in range(shape[self.orth_axis]):
                px = read_bmp("%s%d-%s.bmp" % (base, s, tag))
                idx = [slice(None)] * 3
                idx[self.orth_axis] = s
                out[tuple(idx)] = inv(px, vmin, vmax)
            return torch.from_numpy(out)
        px = read_bmp("%s-%s.bmp" % (base, tag))
        return torch.from_numpy(inv(px, vmin, vmax).reshape(shape))
