"""Readiness-aware gradient bucket plan ("Overlap analysis").

The reference exchanges the whole accumulated gradient in one blocking star round trip
after backward (ref.py:264 gather, ref.py:396 broadcast): nothing overlaps.  Here buckets
are all-reduced from backward as soon as their last gradient is written, so the exposed
communication is only what is still in flight when backward ends.  Where the bucket cuts
sit decides that: U-Net backward produces most gradient BYTES in the deep layers (the
middle of backward), while the high-resolution encoder layers — the last ~20% of backward
compute — produce only the last few percent of the bytes.  A size-only cut can leave a big
deep-layer bucket waiting for one high-resolution tensor and finishing after backward.

Model (per optimizer step, one rank):

* ``ready[i]``: when parameter i's gradient is complete, as a fraction of backward compute —
  backward runs the modules in reverse forward order, a conv costs 2x its forward MACs
  (data + weight gradient), BatchNorm / ReLU / pooling ~0; a module's parameters are ready
  when its backward is done;
* collectives run one after another on the communication stream: a bucket starts at
  max(its last gradient ready, the previous bucket done) and takes
  ``latency + 2 (W-1)/W * bytes / bandwidth`` (ring all-reduce; xGMI is point-to-point, so a
  ring is per-link bound: 7 links x ~153 GB/s per MI355X, of which one ring uses one);
* the plan minimises the time the last bucket finishes plus a small per-bucket charge by
  dynamic programming over contiguous cuts of the flat gradient (buckets are zero-copy
  slices of it, ``parallel/flat.py``), each bucket at most ``cap_bytes`` unless it is one
  tensor.  For the flagship config (256², width/2, 8 ranks) that is five deep buckets of
  4-8 MB that finish 1-7 ms before backward ends and a 40 KB tail (down_conv1) — the
  size-only cut leaves a 15 MB bucket that waits for down_conv2..1.

The flat order is backward order (reverse registration), so readiness is non-decreasing
along it and a bucket is ready when its last parameter is.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

# ring all-reduce model defaults (per-link bound ring over xGMI; RCCL small-message latency)
XGMI_RING_GBPS = 120.0
XGMI_LAT_US = 40.0
# gloo over loopback TCP (the CPU rehearsal)
GLOO_GBPS = 1.0
GLOO_LAT_US = 300.0


def backward_readiness(model_cfg, tile: int, names: Sequence[str]) -> List[float]:
    """Fraction of backward compute done when each named parameter's gradient is complete.
    ``names``: parameter names of ``models.UNet`` (any order); computed on a meta-device copy
    (no memory, no kernels)."""
    from ..models.unet import UNet
    with torch.device("meta"):
        model = UNet.from_config(model_cfg)
    probe = 2 ** model_cfg.depth * 2
    order: List[Tuple[str, float]] = []          # (module name, backward cost) in forward order
    mod_name = {m: n for n, m in model.named_modules()}

    def hook(mod, inp, out):
        cost = 0.0
        if isinstance(mod, (nn.Conv2d, nn.Conv3d)):
            k = 1
            for s in mod.kernel_size:
                k *= s
            cost = 2.0 * out.numel() * (mod.in_channels // mod.groups) * k
        elif isinstance(mod, (nn.ConvTranspose2d, nn.ConvTranspose3d)):
            cost = 2.0 * out.numel() * mod.in_channels
        order.append((mod_name[mod], cost))

    leaves = [m for m in model.modules() if any(True for _ in m.parameters(recurse=False))]
    hs = [m.register_forward_hook(hook) for m in leaves]
    with torch.no_grad():
        model(torch.empty((1, model_cfg.in_channels) + (probe,) * model_cfg.dims, device="meta"))
    for h in hs:
        h.remove()
    total = sum(c for _, c in order) or 1.0
    done, ready_of = 0.0, {}
    for name, cost in reversed(order):            # backward: reverse forward order
        done += cost
        ready_of[name] = done / total
    out = []
    for n in names:
        mod = n.rsplit(".", 1)[0] if "." in n else ""
        out.append(ready_of.get(mod, 1.0))
    return out


@dataclass
class BucketPlan:
    cuts: List[int]                  # bucket k = params [cuts[k], cuts[k+1]) of the flat order
    finish_ms: float                 # predicted time the last bucket's collective ends
    backward_ms: float               # predicted backward time
    bucket_done_ms: List[float]      # predicted end of each bucket's collective
    calibrated: bool = False         # readiness / backward time measured (Trainer.calibrate_bucket_plan)

    @property
    def exposed_ms(self) -> float:
        return max(0.0, self.finish_ms - self.backward_ms)


def _simulate(bounds: Sequence[int], nbytes: Sequence[float], ready_ms: Sequence[float],
              coll_ms) -> List[float]:
    t, out = 0.0, []
    for a, b in zip(bounds[:-1], bounds[1:]):
        start = max(t, max(ready_ms[a:b]))
        t = start + coll_ms(sum(nbytes[a:b]))
        out.append(t)
    return out


def plan_buckets(nbytes: Sequence[float], ready_frac: Sequence[float], backward_ms: float,
                 world: int, gbps: float, lat_us: float, cap_bytes: float,
                 max_buckets: int = 16) -> BucketPlan:
    """Optimal contiguous bucket cuts under the serial-collective model (module docstring):
    for every bucket count k <= ``max_buckets`` the cuts with the earliest final finish
    (dynamic programming over (parameters, buckets)), then the k minimising finish + k x a
    quarter of the collective latency (each extra collective costs a launch and CUs beside
    backward even when the model hides it)."""
    n = len(nbytes)
    ready_ms = [r * backward_ms for r in ready_frac]
    f = 2.0 * (world - 1) / max(world, 1)

    def coll_ms(b):
        return lat_us * 1e-3 + f * b / (gbps * 1e6)

    INF = float("inf")
    # (at least the greedy size cut's count + 2, so a small cap always has a feasible plan)
    K = max(1, min(n, max(max_buckets, len(size_plan_cuts(nbytes, cap_bytes)) + 1)))
    # fin[k][i]: earliest finish of the first i params in exactly k buckets
    fin = [[INF] * (n + 1) for _ in range(K + 1)]
    arg = [[0] * (n + 1) for _ in range(K + 1)]
    fin[0][0] = 0.0
    spans = []                                   # (j, i, size, ready) for every legal bucket
    for i in range(1, n + 1):
        size, rmax = 0.0, 0.0
        for j in range(i - 1, -1, -1):
            size += nbytes[j]
            rmax = max(rmax, ready_ms[j])
            if size > cap_bytes and j < i - 1:
                break
            spans.append((j, i, size, rmax))
    by_end: Dict[int, List[Tuple[int, float, float]]] = {}
    for j, i, size, rmax in spans:
        by_end.setdefault(i, []).append((j, size, rmax))
    for k in range(1, K + 1):
        prev, cur, a = fin[k - 1], fin[k], arg[k]
        for i in range(1, n + 1):
            for j, size, rmax in by_end.get(i, ()):
                fj = prev[j]
                if fj == INF:
                    continue
                t = max(rmax, fj) + coll_ms(size)
                if t < cur[i]:
                    cur[i], a[i] = t, j
    penalty = 0.25 * lat_us * 1e-3
    kbest = min((k for k in range(1, K + 1) if fin[k][n] < INF),
                key=lambda k: (fin[k][n] + penalty * k, k))
    cuts, i = [n], n
    for k in range(kbest, 0, -1):
        i = arg[k][i]
        cuts.append(i)
    cuts.reverse()
    done = _simulate(cuts, nbytes, ready_ms, coll_ms)
    return BucketPlan(cuts=cuts, finish_ms=done[-1] if done else 0.0, backward_ms=backward_ms,
                      bucket_done_ms=done)


def fit_collective_model(nbytes: Sequence[float], ms: Sequence[float],
                         world: int) -> Optional[Tuple[float, float]]:
    """Least-squares fit of ``ms = lat + 2 (W-1)/W * bytes / bandwidth`` to measured
    collectives -> (GB/s, latency us); None without two distinct sizes or for a
    non-physical fit."""
    pts = [(float(b), float(t)) for b, t in zip(nbytes, ms) if b > 0 and t > 0]
    if len({b for b, _ in pts}) < 2:
        return None
    f = 2.0 * (world - 1) / max(world, 1)
    xs = [f * b for b, _ in pts]
    ys = [t for _, t in pts]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    if sxx <= 0:
        return None
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx      # ms per byte
    lat_ms = max(0.0, my - slope * mx)
    if slope <= 0:
        return None
    return 1.0 / (slope * 1e6), lat_ms * 1e3


def size_plan_cuts(nbytes: Sequence[float], cap_bytes: float) -> List[int]:
    """The size-only cuts (``GradBucketReducer``'s original rule), for comparison."""
    cuts, cur = [0], 0.0
    for i, b in enumerate(nbytes):
        if cur and cur + b > cap_bytes:
            cuts.append(i)
            cur = 0.0
        cur += b
    cuts.append(len(nbytes))
    return cuts


def evaluate_cuts(cuts: Sequence[int], nbytes, ready_frac, backward_ms, world, gbps,
                  lat_us) -> BucketPlan:
    f = 2.0 * (world - 1) / max(world, 1)
    ready_ms = [r * backward_ms for r in ready_frac]
    done = _simulate(cuts, nbytes, ready_ms,
                     lambda b: lat_us * 1e-3 + f * b / (gbps * 1e6))
    return BucketPlan(cuts=list(cuts), finish_ms=done[-1] if done else 0.0,
                      backward_ms=backward_ms, bucket_done_ms=done)


def plan_for_model(model: nn.Module, order: Sequence[torch.nn.Parameter], model_cfg, tile: int,
                   batch: int, world: int, backend: Optional[str], cap_mb: float,
                   wire_bytes: int = 4, rate_tflops: Optional[float] = None,
                   gbps: Optional[float] = None, lat_us: Optional[float] = None) -> BucketPlan:
    """The readiness-aware plan for ``order`` (the flat gradient's parameter order)."""
    from ..utils.flops import unet_train_flops_per_sample
    names_of: Dict[int, str] = {id(p): n for n, p in model.named_parameters()}
    names = [names_of[id(p)] for p in order]
    ready = backward_readiness(model_cfg, tile, names)
    gpu = backend == "nccl"
    if rate_tflops is None:
        rate_tflops = 600.0 if gpu else 0.2     # measured step rates: HIP engine / CPU eager
    if gbps is None:
        gbps = XGMI_RING_GBPS if gpu else GLOO_GBPS
    if lat_us is None:
        lat_us = XGMI_LAT_US if gpu else GLOO_LAT_US
    bwd_flop = 2.0 / 3.0 * unet_train_flops_per_sample(model_cfg, tile) * batch
    backward_ms = bwd_flop / (rate_tflops * 1e12) * 1e3
    nbytes = [float(p.numel() * wire_bytes) for p in order]
    return plan_buckets(nbytes, ready, backward_ms, max(world, 2), gbps, lat_us,
                        cap_mb * (1 << 20) * wire_bytes / 4.0)
