"""Datasets: the Vaihingen directory convention and a synthetic Vaihingen-shape generator.

Reference behaviour (ref.py:660-674, ref.py:737-741):

* ``load_files(path)`` walks ``sorted(os.listdir(path))``; files whose name contains
  ``.npy`` are label maps (``np.load``), every other file is an image
  (``imageio.imread``).  Labels are cast to ``uint8``.  The LAST 30 pairs form the test
  split (never evaluated in the reference; ``validate()`` uses it here).
* Images are ``float32 / 255`` and transposed to NCHW; labels become ``int64``.

The reference hard-codes 127 tiles of 512x512 and re-reads the directory every epoch
(ref.py:732); here the directory is read once and the tile size comes from the data.

The synthetic generator (the benchmark data source; there is no network for the real
ISPRS Vaihingen set) produces learnable tiles of the same shape: piecewise-constant
6-class label maps from a coarse random grid, rendered with a per-class colour plus
noise, seeded per sample index so every rank and every run sees the same sample ``i``.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np
import torch

# ISPRS Vaihingen palette order (impervious, building, low veg, tree, car, clutter).
_PALETTE = np.array([[255, 255, 255], [0, 0, 255], [0, 255, 255],
                     [0, 255, 0], [255, 255, 0], [255, 0, 0]], dtype=np.float32) / 255.0


def _read_image(path: str) -> np.ndarray:
    if path.endswith(".npy"):
        return np.load(path)          # allow_pickle=False (default)
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


def load_files(path: str, test_holdout: int = 30
               ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Reference-compatible directory loader (ref.py:660-674).

    Returns ``x_train, y_train, x_test, y_test`` with images as uint8 HWC and labels uint8.
    Label files are recognised by ``'.npy' in name`` exactly as the reference does; image
    files may be any PIL-readable format.  (The reference uses ``imageio``; it is not
    installed here, PIL reads the same PNG/TIFF tiles.)
    """
    xs: List[np.ndarray] = []
    ys: List[np.ndarray] = []
    for name in sorted(os.listdir(path)):
        full = os.path.join(path, name)
        if ".npy" in name:
            ys.append(np.load(full))
        else:
            xs.append(_read_image(full))
    x = np.array(xs)
    y = np.array(ys, dtype="uint8")
    if len(x) != len(y):
        raise ValueError(f"{path}: {len(x)} images but {len(y)} label files")
    if test_holdout > 0:
        return x[:-test_holdout], y[:-test_holdout], x[-test_holdout:], y[-test_holdout:]
    return x, y, x[:0], y[:0]


def to_tensors(x: np.ndarray, y: np.ndarray) -> Tuple[torch.Tensor, torch.Tensor]:
    """uint8 NHWC -> float32 NCHW in [0,1]; labels -> int64 (ref.py:737,741)."""
    xt = torch.from_numpy(np.ascontiguousarray(x)).float().div_(255.0)
    xt = xt.permute(0, 3, 1, 2).contiguous()
    return xt, torch.from_numpy(y.astype("int64"))


class TileDataset:
    """In-memory (image, label) tiles; images NCHW float32, labels int64."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor):
        assert x.shape[0] == y.shape[0]
        self.x, self.y = x, y

    def __len__(self):
        return self.x.shape[0]

    def get(self, idx) -> Tuple[torch.Tensor, torch.Tensor]:
        idx = torch.as_tensor(idx, dtype=torch.long)
        return self.x[idx], self.y[idx]

    @classmethod
    def from_dir(cls, path: str, test_holdout: int = 30):
        xtr, ytr, xte, yte = load_files(path, test_holdout)
        return cls(*to_tensors(xtr, ytr)), cls(*to_tensors(xte, yte)) if len(xte) else None


class SyntheticTiles:
    """Deterministic synthetic Vaihingen-shape tiles (RGB, ``classes`` labels).

    ``get(indices)`` renders the requested samples; sample ``i`` depends only on
    ``(seed, i)``.  Works for 2-D tiles (``dims=2``: [N,3,T,T]) and 3-D volumes
    (``dims=3``: [N,C,T,T,T]).  ``device`` lets the GPU render batches directly in HBM.
    """

    def __init__(self, length: int, tile: int, classes: int = 6, in_channels: int = 3,
                 seed: int = 0, dims: int = 2, grid: int = 8, noise: float = 0.15,
                 device: Optional[torch.device] = None):
        self.length, self.tile, self.classes = length, tile, classes
        self.in_channels, self.seed, self.dims = in_channels, seed, dims
        self.grid, self.noise = max(1, min(grid, tile)), noise
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        pal = _PALETTE
        if classes > len(pal) or in_channels != 3:
            g = np.random.default_rng(1234)
            pal = g.random((classes, in_channels), dtype=np.float32)
        self.palette = torch.tensor(pal[:classes, :in_channels], dtype=torch.float32)

    def __len__(self):
        return self.length

    def _sample(self, i: int):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(i))
        sp = (self.grid,) * self.dims
        coarse = torch.randint(0, self.classes, (1, 1) + sp, generator=g).float()
        full = torch.nn.functional.interpolate(coarse, size=(self.tile,) * self.dims,
                                               mode="nearest")[0, 0].long()
        img = self.palette[full]                                   # [..., C]
        img = img + self.noise * torch.randn(img.shape, generator=g)
        img = img.clamp_(0.0, 1.0)
        perm = (self.dims,) + tuple(range(self.dims))
        return img.permute(*perm).contiguous(), full

    def get(self, idx) -> Tuple[torch.Tensor, torch.Tensor]:
        idx = [int(i) for i in torch.as_tensor(idx).reshape(-1).tolist()]
        xs, ys = zip(*(self._sample(i) for i in idx))
        x = torch.stack(xs).to(self.device, non_blocking=True)
        y = torch.stack(ys).to(self.device, non_blocking=True)
        return x, y


def device_random_batch(batch: int, tile: int, classes: int, device, in_channels: int = 3,
                        dims: int = 2, channels_last: bool = True, dtype=torch.bfloat16,
                        seed: int = 0):
    """A benchmark batch rendered directly on the device (no host round trip).

    Returns the image in the layout the HIP path consumes (NHWC/NDHWC memory, bf16) as an
    NCHW-shaped view, plus int64 labels.  Same generator recipe as ``SyntheticTiles``
    (coarse random label grid, palette colour + noise) so DVFS sees realistic data.
    """
    g = torch.Generator(device=device).manual_seed(seed)
    sp = (8,) * dims
    coarse = torch.randint(0, classes, (batch, 1) + sp, generator=g, device=device).float()
    lab = torch.nn.functional.interpolate(coarse, size=(tile,) * dims, mode="nearest")[:, 0].long()
    pal = torch.rand(classes, in_channels, generator=g, device=device)
    img = pal[lab] + 0.15 * torch.randn(lab.shape + (in_channels,), generator=g, device=device)
    img = img.clamp_(0, 1).to(dtype)                                # N,spatial...,C contiguous
    perm = (0, dims + 1) + tuple(range(1, dims + 1))
    x = img.permute(*perm)                                          # NCHW view of NHWC memory
    if not channels_last:
        x = x.contiguous()
    return x, lab
