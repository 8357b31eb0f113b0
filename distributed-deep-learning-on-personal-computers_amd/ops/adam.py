"""Flat fused Adam (K14 of SURVEY.md §2.5).

Reference: ``torch.optim.Adam(model.parameters())`` at defaults (lr 1e-3, betas
(0.9, 0.999), eps 1e-8, no weight decay; ref.py:704), stepped on every rank with identical
gradients (ref.py:437,552).  The reference ships the live Adam object to the workers by
pickle (ref.py:561); here each rank builds its own from the same config.

Implementation: parameters, gradients and both moments live in flat fp32 buffers
(``parallel.flat.FlatParams``).  On GPU one HIP launch (``adam_step`` in
``csrc/misc.hip``) updates the whole model — 8.7 M elements, 4 streams read + 3 written,
HBM-bound — and, when a weight-pack table is attached, ALSO writes the bf16 copies of the
conv weights in the layouts the conv kernels consume (KRSC for forward, flipped CRSK for
dgrad), so no separate cast/transpose pass runs before the next forward.  On CPU the
same update is a handful of vectorised torch ops on the flat buffers.

``state_dict()`` is format-compatible with ``torch.optim.Adam`` (per-parameter ``step``,
``exp_avg``, ``exp_avg_sq``), so checkpoints load into either optimizer.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from . import _ext


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, flat, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, use_hip: Optional[bool] = None):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        amsgrad=False, maximize=False, foreach=None, capturable=False,
                        differentiable=False, fused=None)
        self.flat = flat
        super().__init__(flat.params, defaults)
        dev = flat.param_buf.device
        self.exp_avg = torch.zeros_like(flat.param_buf)
        self.exp_avg_sq = torch.zeros_like(flat.param_buf)
        self.step_count = 0
        self._bind_state()
        self.weight_pack = None          # set by ops.fused_unet (bf16 conv-weight copies)
        self._dev_scal = None            # device [t, step_size, inv_sqrt_bc2] (hipGraph mode)
        self._use_hip = (dev.type == "cuda") if use_hip is None else use_hip
        if self._use_hip:
            _ext.ops()                   # fail loudly if the kernel library is missing
            # bias corrections on the device: identical arithmetic for eager and hipGraph
            # steps, and nothing step-dependent is baked into a captured graph
            self.enable_device_scalars()

    def _bind_state(self):
        for p in self.flat.params:
            a, b = self.flat.span(p)
            st = self.state[p]
            st["step"] = torch.tensor(float(self.step_count))
            st["exp_avg"] = self.flat._view(self.exp_avg, a, p)
            st["exp_avg_sq"] = self.flat._view(self.exp_avg_sq, a, p)

    def enable_device_scalars(self):
        """Bias corrections computed ON the device (adam_step_dev), so a captured step
        replays correctly: no host scalar is baked into the graph."""
        if not self._use_hip:
            raise RuntimeError("device-side Adam scalars need the HIP kernel library")
        self._dev_scal = torch.tensor([float(self.step_count), 0.0, 0.0],
                                      dtype=torch.float32, device=self.flat.param_buf.device)

    def note_replayed_step(self):
        """Host mirror of a step executed by a graph replay."""
        self.step_count += 1

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        self.step_count += 1
        P, G = self.flat.param_buf, self.flat.grad_buf
        if self._dev_scal is not None:
            _ext.ops().adam_step_dev(P, G, self.exp_avg, self.exp_avg_sq, self._dev_scal,
                                     float(lr), float(b1), float(b2), float(eps), float(wd))
            if self.weight_pack is not None:
                self.weight_pack()
            return loss
        t = self.step_count
        bc1 = 1.0 - b1 ** t
        bc2 = 1.0 - b2 ** t
        step_size = lr / bc1
        inv_sqrt_bc2 = 1.0 / math.sqrt(bc2)
        if self._use_hip:
            _ext.ops().adam_step(P, G, self.exp_avg, self.exp_avg_sq, float(b1), float(b2),
                                 float(eps), float(wd), float(step_size), float(inv_sqrt_bc2))
            if self.weight_pack is not None:
                self.weight_pack()
        else:
            grad = G if wd == 0 else G.add(P, alpha=wd)
            self.exp_avg.lerp_(grad, 1.0 - b1)
            self.exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1.0 - b2)
            denom = (self.exp_avg_sq.sqrt() * inv_sqrt_bc2).add_(eps)
            P.addcdiv_(self.exp_avg, denom, value=-step_size)
        return loss

    def _sync_steps(self):
        for p in self.flat.params:
            self.state[p]["step"].fill_(float(self.step_count))

    def state_dict(self):
        self._sync_steps()       # per-parameter step counters are refreshed lazily
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = []
        with torch.no_grad():
            for p in self.flat.params:
                st = self.state.get(p, {})
                a, b = self.flat.span(p)
                if "exp_avg" in st:
                    self.flat._view(self.exp_avg, a, p).copy_(st["exp_avg"])
                    self.flat._view(self.exp_avg_sq, a, p).copy_(st["exp_avg_sq"])
                if "step" in st:
                    steps.append(int(float(st["step"])))
        self.step_count = max(steps) if steps else 0
        if self._dev_scal is not None:
            self._dev_scal[0] = float(self.step_count)
        self._bind_state()
        if self.weight_pack is not None:
            self.weight_pack()
