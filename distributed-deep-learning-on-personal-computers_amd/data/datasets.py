"""Datasets: the Vaihingen directory convention and a synthetic Vaihingen-shape generator.

Reference behaviour (ref.py:660-674, ref.py:737-741):

* ``load_files(path)`` walks ``sorted(os.listdir(path))``; files whose name contains
  ``.npy`` are label maps (``np.load``), every other file is an image
  (``imageio.imread``).  Labels are cast to ``uint8``.  The LAST 30 pairs form the test
  split (never evaluated in the reference; ``validate()`` uses it here).
* Images are ``float32 / 255`` and transposed to NCHW; labels become ``int64``.

The reference hard-codes 127 tiles of 512x512, re-reads the directory every epoch
(ref.py:732) and copies every micro-batch from the host (ref.py:754-755).  Here:

* the directory is read once; ``TileDataset`` keeps the raw uint8 NHWC tiles and, on a GPU,
  ``to_device()`` uploads them ONCE to HBM (288 GB: the reference's 127 tiles of 512² are
  100 MB), after which a batch is one gather kernel (``tile_gather``: /255, channel-last
  bf16 padded to 8 channels, int64 labels — SURVEY.md K20).  Datasets too large for the
  HBM budget stay in pinned host memory and are prefetched one batch ahead on a copy
  stream;
* the synthetic generator (the benchmark data source; there is no network for the real
  ISPRS Vaihingen set) renders learnable tiles of the same shape — piecewise-constant
  class maps from a coarse random lattice, a per-class colour plus noise — from a
  counter-based hash of ``(seed, sample index, pixel)``.  On the HIP path a batch is ONE
  kernel writing the first conv's input layout straight into HBM (``csrc/data.hip``);
  ``render_synthetic`` is the bit-identical PyTorch twin (CPU tests, ``impl="torch"``).
  Sample ``i`` never depends on which rank, batch slot or resume point renders it.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import numpy as np
import torch

# ISPRS Vaihingen palette order (impervious, building, low veg, tree, car, clutter).
_PALETTE = np.array([[255, 255, 255], [0, 0, 255], [0, 255, 255],
                     [0, 255, 0], [255, 255, 0], [255, 0, 0]], dtype=np.float32) / np.float32(255.0)

_M32 = 0xFFFFFFFF


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


# ---------------------------------------------------------------------- engine input layout
def engine_input(x_nhwc: torch.Tensor, in_channels: int) -> torch.Tensor:
    """Wrap a channel-last bf16 batch whose channels are zero-padded (to 8) as the NCHW-shaped
    view the model API takes.  The HIP engine recognises the attached padded tensor and uses
    it as the first conv's input with no conversion pass; any other consumer sees an ordinary
    [N, C, (D,) H, W] tensor."""
    nd = x_nhwc.dim()
    v = x_nhwc[..., :in_channels].permute(0, nd - 1, *range(1, nd - 1))
    v._ddlpc_nhwc = x_nhwc
    return v


def split_batch(x: torch.Tensor, y: torch.Tensor, n: int) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """A batch rendered in one pass (e.g. a whole accumulation window) as ``n`` equal
    micro-batches that are zero-copy views of it (engine-layout inputs keep their layout),
    so the trainer's batched window (``Trainer._cat_window``) can take the batch back
    without a copy."""
    if x.shape[0] % n:
        raise ValueError(f"batch of {x.shape[0]} does not split into {n} equal micro-batches")
    b = x.shape[0] // n
    xp = getattr(x, "_ddlpc_nhwc", None)
    out = []
    for i in range(n):
        xi = engine_input(xp[i * b:(i + 1) * b], x.shape[1]) if xp is not None else x[i * b:(i + 1) * b]
        out.append((xi, y[i * b:(i + 1) * b]))
    return out


def cat_adjacent(ts: List[torch.Tensor]) -> torch.Tensor:
    """torch.cat along dim 0 — without a copy when the tensors are contiguous, equal-shaped
    and lie back to back in one storage (the views ``split_batch`` hands out)."""
    t0 = ts[0]
    step = t0.numel()
    ok = all(t.is_contiguous() and t.shape == t0.shape and t.dtype == t0.dtype and
             t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr() and
             t.storage_offset() == t0.storage_offset() + i * step for i, t in enumerate(ts))
    if not ok or t0.dim() == 0:
        return torch.cat(ts)
    # (explicit contiguous strides: is_contiguous() ignores the stride of a size-1 dim, so a
    # batch-1 micro-batch may carry any stride[0])
    shape = (t0.shape[0] * len(ts),) + tuple(t0.shape[1:])
    strides, acc = [], 1
    for d in reversed(shape):
        strides.append(acc)
        acc *= d
    out = t0.new_empty(0)
    out.set_(t0.untyped_storage(), t0.storage_offset(), shape, tuple(reversed(strides)))
    return out


class DevicePrefetcher:
    """Device-side input pipeline: ``get(k)`` returns batch k (``make(k)``) and starts
    rendering batch k + 1 on a side HIP stream, so the generator / gather kernels of the next
    step run under this step's compute instead of in front of it (every batch is still
    rendered, one per step).  The current stream waits on the batch's event, and every tensor
    of the batch is recorded on it, so the caching allocator never hands the memory back to
    the side stream while the step may still read it."""

    def __init__(self, make, device):
        self.make = make
        self.stream = torch.cuda.Stream(torch.device(device))
        self.pending = {}

    def _launch(self, k):
        # (no wait on the current stream: the render reads nothing the step writes)
        with torch.cuda.stream(self.stream):
            batch = self.make(k)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.pending[k] = (batch, ev)

    @staticmethod
    def _tensors(obj):
        if isinstance(obj, torch.Tensor):
            yield obj
            base = getattr(obj, "_ddlpc_nhwc", None)
            if base is not None:
                yield base
        elif isinstance(obj, (list, tuple)):
            for o in obj:
                yield from DevicePrefetcher._tensors(o)

    def get(self, k):
        if k not in self.pending:
            self.pending.clear()
            self._launch(k)
        batch, ev = self.pending.pop(k)
        cur = torch.cuda.current_stream(self.stream.device)
        cur.wait_event(ev)
        for t in self._tensors(batch):
            t.record_stream(cur)
        self._launch(k + 1)
        return batch

    def get_last(self, k):
        """``get(k)`` without starting batch k + 1 (the end of the index list)."""
        if k not in self.pending:
            self.pending.clear()
            self._launch(k)
        batch, ev = self.pending.pop(k)
        cur = torch.cuda.current_stream(self.stream.device)
        cur.wait_event(ev)
        for t in self._tensors(batch):
            t.record_stream(cur)
        return batch


# ---------------------------------------------------------------------- synthetic tiles
def device_indices(idx, device) -> torch.Tensor:
    """Sample indices as an int64 tensor on ``device`` without a blocking host round trip:
    a device tensor is used as is; host indices go through pinned memory, so the
    host->device copy is asynchronous (a pageable copy, or ``.tolist()`` of a device
    tensor, would stall the host until the GPU drained its queue — measured 0.6 ms of idle
    GPU per training step)."""
    device = torch.device(device)
    if torch.is_tensor(idx) and idx.device.type == device.type:
        return idx.reshape(-1).to(torch.int64)
    it = torch.as_tensor(idx, dtype=torch.int64).reshape(-1)
    if device.type == "cuda":
        return it.pin_memory().to(device, non_blocking=True)
    return it.to(device)


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 integer hash on int64 tensors holding uint32 values (== csrc/data.hip)."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def _mix32_int(v: int) -> int:
    v &= _M32
    v ^= v >> 16
    v = (v * 0x7FEB352D) & _M32
    v ^= v >> 15
    v = (v * 0x846CA68B) & _M32
    return v ^ (v >> 16)


def synthetic_palette(classes: int, in_channels: int) -> torch.Tensor:
    """Per-class colours: the Vaihingen palette for <= 6 RGB classes, else hashed colours."""
    if classes <= len(_PALETTE) and in_channels == 3:
        return torch.from_numpy(_PALETTE[:classes].copy())
    pal = np.empty((classes, in_channels), dtype=np.float32)
    for k in range(classes):
        for c in range(in_channels):
            h = _mix32_int(0x5BD1E995 ^ _mix32_int(k * 16 + c))
            pal[k, c] = np.float32(h >> 8) * np.float32(1.0 / 16777216.0)
    return torch.from_numpy(pal)


def noise_k(noise: float) -> float:
    """fp32 scale of the Irwin-Hall noise (std ``noise``), rounded once, shared host/device."""
    return float(np.float32(noise * math.sqrt(3.0)))


def render_synthetic(idx, seed: int, classes: int, in_channels: int, tile: int, dims: int,
                     grid: int = 8, noise: float = 0.15, device=None,
                     palette: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """PyTorch twin of ``synth_tiles_kernel``: the same bits, NCHW float32 + int64 labels."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    idx = torch.as_tensor(idx, dtype=torch.int64).reshape(-1).to(device)
    B = idx.numel()
    pal = (palette if palette is not None else synthetic_palette(classes, in_channels)).to(device)
    ar = torch.arange(tile, device=device, dtype=torch.int64)
    cg = (ar * grid) // tile                                    # nearest lattice cell
    if dims == 2:
        cell = cg[:, None] * grid + cg[None, :]
    else:
        cell = (cg[:, None, None] * grid + cg[None, :, None]) * grid + cg[None, None, :]
    S = tile ** dims
    skey = _mix32_int(seed ^ 0x9E3779B9)
    key = _mix32(torch.full_like(idx, skey) ^ (idx & _M32))     # [B]
    ckey = _mix32((cell.reshape(-1) + 0x632BE5AB) & _M32)       # [S]
    lab = _mix32(key[:, None] ^ ckey[None, :]) % classes         # [B, S]
    p = torch.arange(S, device=device, dtype=torch.int64)
    xs = []
    inv = torch.tensor(1.0 / 16777216.0, dtype=torch.float32, device=device)
    k = torch.tensor(noise_k(noise), dtype=torch.float32, device=device)
    for c in range(in_channels):
        base = key[:, None] ^ _mix32((p * 8 + c + 0x1B873593) & _M32)[None, :]
        s = None
        for j in range(4):
            u = (_mix32((base + j * 0x9E3779B9) & _M32) >> 8).to(torch.float32) * inv
            s = u if s is None else s + u
        n = (s - 2.0) * k
        xs.append((pal[lab, c] + n).clamp_(0.0, 1.0))
    x = torch.stack(xs, 1).reshape((B, in_channels) + (tile,) * dims)
    return x, lab.reshape((B,) + (tile,) * dims)


class SyntheticTiles:
    """Deterministic synthetic Vaihingen-shape tiles (``classes`` labels, ``in_channels``).

    ``get(indices)`` renders the requested samples; sample ``i`` depends only on
    ``(seed, i)``.  2-D tiles (``dims=2``: [N,C,T,T]) or 3-D volumes (``dims=3``).
    ``device``/``layout`` select where and how a batch is produced:

    * ``layout="nchw"`` (default): float32 NCHW via ``render_synthetic``, the PyTorch twin
      (stock-op path), on the CPU or a GPU;
    * ``layout="engine"``: one ``synth_tiles`` operator call writes the engine's input
      (channel-last bf16, 8 channels) — the HIP kernel into HBM on a GPU, its C++ twin
      (csrc/cpu_ref.cpp, the same bits) on the CPU; see ``engine_input``.
    """

    def __init__(self, length: int, tile: int, classes: int = 6, in_channels: int = 3,
                 seed: int = 0, dims: int = 2, grid: int = 8, noise: float = 0.15,
                 device: Optional[torch.device] = None, layout: str = "nchw"):
        if layout not in ("nchw", "engine"):
            raise ValueError(f"layout={layout!r}")
        self.length, self.tile, self.classes = length, tile, classes
        self.in_channels, self.seed, self.dims = in_channels, seed, dims
        self.grid, self.noise = max(1, min(grid, tile)), noise
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.layout = layout
        self.palette = synthetic_palette(classes, in_channels).to(self.device)

    def __len__(self):
        return self.length

    @property
    def on_device(self) -> bool:
        """Batches are rendered by a device kernel (``Trainer.fit`` prefetches them)."""
        return self.device.type == "cuda"

    def get(self, idx) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.layout == "engine":
            from ..ops import _ext
            it = device_indices(idx, self.device)
            xp, y = _ext.ops().synth_tiles(it, self.seed, self.classes, self.in_channels,
                                           self.tile, self.dims, self.grid,
                                           noise_k(self.noise), self.palette, 8)
            return engine_input(xp, self.in_channels), y
        return render_synthetic(idx, self.seed, self.classes, self.in_channels, self.tile,
                                self.dims, self.grid, self.noise, self.device, self.palette)


# ---------------------------------------------------------------------- real tiles
class TileDataset:
    """In-memory (image, label) tiles: uint8 NHWC images, uint8 label maps.

    ``get`` returns the reference's tensors (float32 NCHW in [0,1], int64 labels) on the
    host.  ``to_device`` moves the raw uint8 tiles to HBM once (or, above ``budget_bytes``,
    to pinned host memory with a one-batch-ahead copy stream) and returns a dataset whose
    ``get`` produces device batches.
    """

    def __init__(self, x: np.ndarray, y: np.ndarray):
        x = np.asarray(x)
        y = np.asarray(y)
        assert x.shape[0] == y.shape[0] and x.ndim == y.ndim + 1
        if x.dtype != np.uint8:
            raise TypeError("TileDataset holds uint8 images (as read from disk)")
        self.x = torch.from_numpy(np.ascontiguousarray(x))
        self.y = torch.from_numpy(np.ascontiguousarray(y.astype(np.uint8)))

    def __len__(self):
        return self.x.shape[0]

    @property
    def in_channels(self) -> int:
        return int(self.x.shape[-1])

    def get(self, idx) -> Tuple[torch.Tensor, torch.Tensor]:
        idx = torch.as_tensor(idx, dtype=torch.long).reshape(-1)
        x = self.x[idx].float().div_(255.0)
        nd = x.dim()
        return x.permute(0, nd - 1, *range(1, nd - 1)).contiguous(), self.y[idx].long()

    def to_device(self, device, layout: str = "engine",
                  budget_bytes: Optional[int] = None) -> "DeviceTileDataset":
        return DeviceTileDataset(self, device, layout, budget_bytes)

    @classmethod
    def from_dir(cls, path: str, test_holdout: int = 30):
        xtr, ytr, xte, yte = load_files(path, test_holdout)
        return cls(xtr, ytr), (cls(xte, yte) if len(xte) else None)


class DeviceTileDataset:
    """``TileDataset`` served from the GPU.

    * resident (raw bytes <= budget, default half the free HBM): the uint8 tiles live in
      HBM; ``get`` = one ``tile_gather`` kernel (``layout="engine"``) or a device gather +
      convert (``layout="nchw"``).  No host copy per step.
    * streamed: pinned host tiles; ``get`` copies the batch's uint8 bytes on a side copy
      stream (the NEXT batch can be prefetched with ``prefetch(idx)``) and converts on the
      device.
    """

    def __init__(self, base: TileDataset, device, layout: str = "engine",
                 budget_bytes: Optional[int] = None):
        self.base = base
        self.device = torch.device(device)
        self.layout = layout
        self.in_channels = base.in_channels
        nbytes = base.x.numel() + base.y.numel()
        if budget_bytes is None:
            free, _ = torch.cuda.mem_get_info(self.device)
            budget_bytes = free // 2
        self.resident = nbytes <= budget_bytes
        if self.resident:
            self.x = base.x.to(self.device)
            self.y = base.y.to(self.device)
        else:
            self.x = base.x.pin_memory()
            self.y = base.y.pin_memory()
            self.copy_stream = torch.cuda.Stream(self.device)
            self._pending = None

    def __len__(self):
        return len(self.base)

    def prefetch(self, idx):
        """Start the host->device copy of a future batch (streamed mode only)."""
        if self.resident:
            return
        key = tuple(int(i) for i in torch.as_tensor(idx).reshape(-1).tolist())
        ii = torch.tensor(key, dtype=torch.long)
        xs = self.x[ii].pin_memory()
        ys = self.y[ii].pin_memory()
        with torch.cuda.stream(self.copy_stream):
            xd = xs.to(self.device, non_blocking=True)
            yd = ys.to(self.device, non_blocking=True)
        self._pending = (key, xd, yd)

    def _fetch_raw(self, idx):
        key = tuple(int(i) for i in torch.as_tensor(idx).reshape(-1).tolist())
        if self._pending is None or self._pending[0] != key:
            self.prefetch(list(key))
        _, xd, yd = self._pending
        self._pending = None
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self.copy_stream)
        xd.record_stream(cur)
        yd.record_stream(cur)
        return xd, yd

    def get(self, idx) -> Tuple[torch.Tensor, torch.Tensor]:
        if not torch.is_tensor(idx) or idx.device.type == "cpu":
            # host indices: range-checked here (device indices are not — that would be a
            # blocking read-back; the gather kernel turns an out-of-range one into a zero
            # image with ignored labels instead of reading outside the dataset)
            ii = torch.as_tensor(idx, dtype=torch.int64).reshape(-1)
            if ii.numel() and (int(ii.min()) < 0 or int(ii.max()) >= len(self)):
                raise IndexError(f"sample index out of range [0, {len(self)}): "
                                 f"{int(ii.min())}..{int(ii.max())}")
        if self.resident:
            src, lab = self.x, self.y
            it = device_indices(idx, self.device)
        else:
            src, lab = self._fetch_raw(idx)
            it = torch.arange(src.shape[0], device=self.device, dtype=torch.int64)
        if self.layout == "engine":
            from ..ops import _ext
            xp, y = _ext.ops().tile_gather(src, lab, it, 8)
            return engine_input(xp, self.in_channels), y
        x = src.index_select(0, it).float().div_(255.0)
        nd = x.dim()
        mf = torch.channels_last if nd == 4 else torch.channels_last_3d
        x = x.permute(0, nd - 1, *range(1, nd - 1)).contiguous(memory_format=mf)
        return x, lab.index_select(0, it).long()


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
