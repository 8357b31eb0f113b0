"""Lossy gradient codec (the reference's ``model_bytes`` compression, ref.py:25,328-545).

Reference formulas (bit-exact here):

* scale   ``max_grad = max over params of max|grad|``   (ref.py:328-340 / 451-463)
* encode  ``q = round(g / max_grad * L)`` cast to fp16 (L = 100) or int8 (L = 10)
          (ref.py:375 / 487 and ref.py:354 / 474)
* decode  ``q.float() / L * max_grad``                 (ref.py:304,313,426,430,533,543)

The reference sends per-tensor byte strings through pickle+mgzip to rank 0 which merges
and re-broadcasts (star).  Here every rank encodes its gradient bucket, the packed
payloads and scales are ``all_gather``-ed, and every rank decodes and sums them in rank
order -> all ranks get bit-identical gradients (the reference achieves that by making the
server also use the decoded copy, ref.py:402-433).

``scale`` granularity: ``global`` (reference parity: one scale over the whole gradient),
``bucket`` (default) or ``tensor``.  A global scale zeroes most small-magnitude tensors
(only 6.4 % non-zeros in fp16 mode on an init-time gradient).

The reference's ``float32`` mode is broken (NameError) and is not offered;
``grad_codec="none"`` is the lossless path.  An all-zero gradient (``max_grad == 0``), a
NameError in the reference, encodes to zeros here.

On GPU the encode is ONE fused HIP kernel pass (absmax reduce + quantize; ``ops.codec``)
and the decode+sum another; this module is the torch oracle used on CPU and in tests.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

LEVELS = {"fp16_absmax": 100.0, "int8_absmax": 10.0}
WIRE_DTYPE = {"fp16_absmax": torch.float16, "int8_absmax": torch.int8}


def absmax(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    m = None
    for t in tensors:
        v = t.detach().abs().max().float()
        m = v if m is None else torch.maximum(m, v)
    return m


def encode(g: torch.Tensor, scale: torch.Tensor, codec: str) -> torch.Tensor:
    """round(g / scale * L) -> wire dtype.  scale == 0 encodes zeros."""
    L = LEVELS[codec]
    safe = torch.where(scale > 0, scale, torch.ones_like(scale))
    q = torch.round(g.float() / safe * L)
    q = torch.where(scale > 0, q, torch.zeros_like(q))
    return q.to(WIRE_DTYPE[codec])


def decode(q: torch.Tensor, scale: torch.Tensor, codec: str) -> torch.Tensor:
    L = LEVELS[codec]
    return q.to(torch.float32) / L * scale


def encode_segments(flat: torch.Tensor, segments: List[Tuple[int, int]], codec: str
                    ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Encode a flat fp32 buffer with one absmax scale per ``(start, end)`` segment.
    Returns (payload in wire dtype, fp32 scales[len(segments)])."""
    scales = torch.stack([flat[a:b].abs().max().float() if b > a else
                          torch.zeros((), device=flat.device) for a, b in segments])
    out = torch.empty(flat.numel(), dtype=WIRE_DTYPE[codec], device=flat.device)
    for (a, b), s in zip(segments, scales):
        out[a:b] = encode(flat[a:b], s, codec)
    return out, scales


def decode_segments_accumulate(acc: torch.Tensor, q: torch.Tensor, scales: torch.Tensor,
                               segments: List[Tuple[int, int]], codec: str,
                               weight: float = 1.0):
    for (a, b), s in zip(segments, scales):
        acc[a:b] += decode(q[a:b], s, codec) * weight


def reference_weights(world_size: int) -> List[float]:
    """Per-rank weights of the reference's "crooked averaging" (ref.py:268-315).

    Rank 0 divides its own grad by M once per worker message and adds each worker's
    decoded grad / M: final = g0 / M^M + sum_j q_j / M^(M-j+1), M = #workers
    (M=1 -> [1, 1] = a SUM; M=2 -> [1/4, 1/4, 1/2]).
    """
    M = world_size - 1
    if M <= 0:
        return [1.0]
    return [M ** (-M)] + [M ** (-(M - j + 1)) for j in range(1, M + 1)]


def relative_l2_error(g: torch.Tensor, codec: str, scale: Optional[torch.Tensor] = None
                      ) -> float:
    s = g.abs().max() if scale is None else scale
    r = decode(encode(g, s, codec), s, codec)
    return float((r - g).norm() / g.norm().clamp_min(1e-30))
