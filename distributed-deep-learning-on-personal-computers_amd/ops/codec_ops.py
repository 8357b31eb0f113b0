"""Gradient codec entry points (K16-K18 of SURVEY.md §2.5).

Three ``torch.ops.ddlpc`` operators, dispatched by tensor device: ``codec_absmax`` (one
multi-segment absmax pass, K16), ``codec_encode`` (quantise to fp16/int8 levels, K17) and
``codec_decode_sum`` (dequantise W payloads, weight and sum in rank order into the fp32
gradient, K18) — the fused HIP kernels of ``csrc/misc.hip`` for GPU tensors, the C++ kernels
of ``csrc/cpu_ref.cpp`` for CPU tensors.  ``parallel.codec`` is the torch oracle both are
tested against (same formulas, bit-exact rounding: round-half-to-even like torch.round).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from . import _ext

CODEC_ID = {"fp16_absmax": 0, "int8_absmax": 1}


def _seg_tensor(segments, device):
    return torch.tensor([x for s in segments for x in s], dtype=torch.int64, device=device)


def encode_segments(flat: torch.Tensor, segments: List[Tuple[int, int]], codec: str
                    ) -> Tuple[torch.Tensor, torch.Tensor]:
    ext = _ext.ops()
    seg = _seg_tensor(segments, flat.device)
    scales = ext.codec_absmax(flat, seg)
    payload = ext.codec_encode(flat, seg, scales, CODEC_ID[codec])
    return payload, scales


def decode_sum_segments(out: torch.Tensor, payloads: Sequence[torch.Tensor],
                        scales: Sequence[torch.Tensor], segments: List[Tuple[int, int]],
                        codec: str, weights: Sequence[float]):
    """out[seg] = sum_r weights[r] * decode(payloads[r][seg], scales[r][k])."""
    ext = _ext.ops()
    seg = _seg_tensor(segments, out.device)
    q = torch.stack(list(payloads))
    s = torch.stack(list(scales))
    w = torch.tensor(list(weights), dtype=torch.float32, device=out.device)
    ext.codec_decode_sum(out, q, s, w, seg, CODEC_ID[codec])
    return out
