"""Flat parameter / gradient storage.

Every parameter becomes a view into ONE contiguous fp32 buffer and every ``.grad`` a view
into ONE contiguous fp32 gradient buffer.  Consequences:

* the gradient all-reduce works on contiguous slices of the flat gradient (buckets are
  zero-copy: SURVEY.md §2.5 K19), instead of the reference's per-tensor byte strings
  (ref.py:358-387);
* the optimizer is one multi-tensor launch over the flat range (K14), and zero_grad is one
  memset (K15);
* the layout is chosen in REVERSE registration order, which is (approximately) the order
  in which backward produces gradients, so buckets complete front to back.

Parameters keep their standard PyTorch shapes/layouts (OIHW conv weights, IOHW transposed
conv weights), so ``state_dict`` stays reference-compatible.
"""
from __future__ import annotations

from typing import List, Tuple

import torch


class FlatParams:
    def __init__(self, params: List[torch.nn.Parameter], reverse: bool = True,
                 align: int = 64):
        self.params = list(params)
        order = list(reversed(self.params)) if reverse else list(self.params)
        self.order = order
        dev = order[0].device
        offs, n = {}, 0
        for p in order:
            offs[id(p)] = n
            n += (p.numel() + align - 1) // align * align     # 256-B aligned views
        self.numel = n
        self.offsets = offs
        self.param_buf = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad_buf = torch.zeros(n, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p in order:
                o = offs[id(p)]
                view = self._view(self.param_buf, o, p)
                view.copy_(p.data.float())
                p.data = view
                p.grad = self._view(self.grad_buf, o, p)

    @staticmethod
    def _view(buf, o, p):
        # keep the parameter's strides (e.g. channels_last conv weights) on the flat buffer
        if p.is_contiguous():
            return buf[o:o + p.numel()].view_as(p)
        return buf.as_strided(p.shape, p.stride(), o)

    def span(self, p) -> Tuple[int, int]:
        o = self.offsets[id(p)]
        return o, o + p.numel()

    def zero_grad(self):
        self.grad_buf.zero_()

    def rebind_grads(self):
        """Re-attach grad views (after something set ``p.grad = None``)."""
        for p in self.order:
            o = self.offsets[id(p)]
            if p.grad is None or p.grad.data_ptr() != self.grad_buf[o:].data_ptr():
                p.grad = self._view(self.grad_buf, o, p)

    def check_bound(self) -> bool:
        for p in self.order:
            o = self.offsets[id(p)]
            if p.data.data_ptr() != self.param_buf[o:].data_ptr():
                return False
        return True


def flatten_module(module: torch.nn.Module, reverse: bool = True) -> FlatParams:
    flat = FlatParams([p for p in module.parameters() if p.requires_grad], reverse=reverse)
    module._flat_params = flat
    return flat
