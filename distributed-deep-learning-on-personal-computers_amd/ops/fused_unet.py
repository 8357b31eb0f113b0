"""The U-Net forward/backward on the hand-written gfx950 kernels (``torch.ops.ddlpc``).

Execution model (SURVEY.md §2.5 kernel inventory -> fusion plan):

* activations are channel-last bf16 tensors of SHAPE [N, (D,) H, W, C]; parameters stay
  fp32 in their reference layouts (the flat fp32 master buffer) and are packed to bf16
  kernel layouts once per optimizer step (``pack_weights``: ONE launch for all convs);
* a ``DoubleConv`` block is ONE autograd node (``_DoubleConvFn``) with an explicit
  backward:

      forward   y1,stats = conv3(x [, skip])            (concat = 2 input pointers)
                s1       = bn_finalize(stats)            (fp64 reduce, running stats)
                y2,stats = conv3(relu(bn1(y1)))          (BN1+ReLU fused in the prologue)
                s2       = bn_finalize(stats)
                a2[,p]   = bn_relu_apply(y2[, pool])     (max-pool fused, encoder only)
      backward  dY2      = bn_backward(da2 [, dpool])    (unpool + skip-sum + ReLU + BN)
                dW2      = conv3_wgrad(dY2, relu(bn1(y1)))   (prologue re-applied)
                dA1      = conv3(dY2, flip(W2)^T)            (data gradient)
                dY1      = bn_backward(dA1)
                dW1      = conv3_wgrad(dY1, x [, skip])
                dx[,dskip] = conv3(dY1, flip(W1)^T) split across the concat inputs

  only x, y1, y2 and the BN statistics are saved; a1 is never materialised and a2 only
  once (it is the skip tensor / next input);
* ``ConvTranspose(2, 2)`` is a GEMM with a pixel-shuffle epilogue (``_ConvTFn``);
* the 1x1 head, softmax cross-entropy, its gradient and the pixel-accuracy count are one
  fused kernel pair (``_HeadCEFn``): logits never reach HBM in training; its backward is
  two passes (stats, then recompute + the last block's BN backward: dA never stored).

Conv biases feeding a training-mode BatchNorm receive an exactly-zero gradient (the BN
mean subtraction cancels them); stock PyTorch returns float noise of ~1e-9 there.
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import _ext

_F = None


def _ops():
    global _F
    if _F is None:
        _F = _ext.ops()
    return _F


def _nhwc_shape_to_nchw(t: torch.Tensor) -> torch.Tensor:
    """View a channel-last [N,(D,)H,W,C] tensor as NCHW (no copy)."""
    nd = t.dim()
    return t.permute(0, nd - 1, *range(1, nd - 1))


class _ConvPack:
    """bf16 kernel-layout copies of one conv / transposed-conv weight."""

    def __init__(self, conv: nn.Module, kind: int, need_dgrad: bool):
        w = conv.weight
        self.conv, self.kind = conv, kind
        dev = w.device
        if kind == 0:                                  # 3x3(x3) conv, OIHW
            cout, cin = w.shape[0], w.shape[1]
            taps = w[0, 0].numel()
            cinw = (cin + 7) // 8 * 8
            self.fwd = torch.zeros(cout, taps, cinw, dtype=torch.bfloat16, device=dev)
            self.dgrad = (torch.zeros(cin, taps, cout, dtype=torch.bfloat16, device=dev)
                          if need_dgrad else None)
            self.shape = (cout, cin, taps, cinw, cout)
        else:                                          # ConvTranspose k2 s2, IOHW
            cin, cout = w.shape[0], w.shape[1]
            taps = w[0, 0].numel()                     # 4 or 8 sub-positions
            self.fwd = torch.zeros(taps * cout, cin, dtype=torch.bfloat16, device=dev)
            self.dgrad = torch.zeros(cin, taps * cout, dtype=torch.bfloat16, device=dev)
            self.shape = (cout, cin, taps, cin, cout)
        self.cout, self.cin, self.taps = self.shape[0], self.shape[1], self.shape[2]

    def entry(self) -> List[int]:
        w = self.conv.weight
        assert w.is_contiguous(), "packed weights need contiguous fp32 parameters"
        cout, cin, taps, cinw, coutw = self.shape
        return [w.data_ptr(), self.fwd.data_ptr(),
                self.dgrad.data_ptr() if self.dgrad is not None else 0,
                (self.kind & 0xffffffff) | (cout << 32), cin | (taps << 32), cinw | (coutw << 32)]

    def numel(self) -> int:
        return self.cout * self.cin * self.taps


class _BNState:
    def __init__(self, bn: nn.Module, engine=None):
        self.bn = bn
        self.engine = engine
        self.index = -1                  # position in engine.bns (deferred running stats)

    def finalize(self, stats_partial: torch.Tensor, count: float) -> torch.Tensor:
        bn = self.bn
        if bn.training:
            mom = bn.momentum if bn.momentum is not None else 0.1
            eng = self.engine
            j = eng.bn_defer_j if eng is not None else None
            if j is not None and bn.track_running_stats:
                # concurrent micro-batch streams: this forward's (mean, unbiased var) go to
                # its own slot (momentum 1 writes them exactly); the momentum updates are
                # applied later in micro-batch order (UNetEngine.bn_defer_apply)
                slot = eng.bn_defer_slot(self.index, j)
                return _ops().bn_finalize(stats_partial, float(count), bn.weight, bn.bias,
                                          slot[0], slot[1], 1.0, float(bn.eps), True, None)
            return _ops().bn_finalize(stats_partial, float(count), bn.weight, bn.bias,
                                      bn.running_mean, bn.running_var, float(mom), float(bn.eps),
                                      bool(bn.track_running_stats), bn.num_batches_tracked)
        return self.eval_stats()

    def finalize_groups(self, y: torch.Tensor, groups: int) -> torch.Tensor:
        """Per-micro-batch statistics of a batched window (``UNetEngine.bn_groups``):
        -> [groups][4][C]; each group's (mean, unbiased var) goes to its row of the engine's
        running-statistics arena, applied in micro-batch order after the forward."""
        bn = self.bn
        eng = self.engine
        arena = eng._bn_arena if (bn.track_running_stats and eng._bn_arena is not None) else None
        off = eng._bn_offs[self.index] if arena is not None else 0
        return _ops().bn_group_finalize(y, groups, bn.weight, bn.bias, float(bn.eps), arena, off)

    def finalize_group_rows(self, rows: torch.Tensor, groups: int, count: float) -> torch.Tensor:
        """``finalize_groups`` from group-major partial rows a conv epilogue wrote
        (``conv3_fwd`` with ``groups``): no statistics pass over y."""
        bn = self.bn
        eng = self.engine
        arena = eng._bn_arena if (bn.track_running_stats and eng._bn_arena is not None) else None
        off = eng._bn_offs[self.index] if arena is not None else 0
        return _ops().bn_group_finalize_rows(rows, groups, float(count), bn.weight, bn.bias,
                                             float(bn.eps), arena, off)

    def eval_stats(self) -> torch.Tensor:
        bn = self.bn
        inv = torch.rsqrt(bn.running_var.float() + bn.eps)
        scale = bn.weight * inv
        shift = bn.bias - bn.running_mean * scale
        return torch.stack([bn.running_mean.float(), inv, scale, shift]).contiguous()


class _DoubleConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x1, x2, w1, b1, g1, be1, w2, b2, g2, be2, blk, pool: bool, defer: bool,
                x2_bn: Optional[torch.Tensor] = None, defer_skip: bool = False):
        # x2_bn: statistics of a deferred skip (x2 = the encoder block's PRE-BN y2): its BN +
        # ReLU is applied on load by the conv / weight-gradient kernels' X2 prologue
        # defer_skip (encoder blocks): hand out the pre-BN y2 as the skip and materialise only
        # the pooled activation
        F = _ops()
        p1, p2 = blk.pack1, blk.pack2
        training = blk.bn1.bn.training
        G = blk.engine.bn_groups if training else 0
        if G >= 1:
            assert not defer_skip and x2_bn is None, "BN groups: no deferred skips"
            return _DoubleConvFn._group_forward(ctx, x1, x2, b1, b2, g1, g2, blk, pool, G, defer)
        ctx.groups = 0
        c1 = p1.cout
        sc2 = x2_bn[2] if x2_bn is not None else None
        sh2 = x2_bn[3] if x2_bn is not None else None
        ctx.x2_bn = x2_bn
        y1, _, st1 = F.conv3_fwd(x1, x2, p1.fwd, b1, None, None, c1, 0, training, sc2, sh2)
        count = float(y1.numel() // c1)
        s1 = blk.bn1.finalize(st1, count) if training else blk.bn1.eval_stats()
        y2, _, st2 = F.conv3_fwd(y1, None, p2.fwd, b2, s1[2], s1[3], p2.cout, 0, training)
        s2 = blk.bn2.finalize(st2, count) if training else blk.bn2.eval_stats()
        ctx.blk = blk
        ctx.pool = pool
        ctx.defer = defer
        # activation recompute: y1 is not kept; backward re-runs conv1 (same kernel, same
        # bits) from the saved inputs.  b1 rides along for that (its own grad stays zero)
        # recompute level 2 also drops y2 when the block hands out a materialised activation
        # (a deferred block's y2 IS its output, held by the consumer anyway)
        rc = int(blk.engine.recompute) if training else 0
        ctx.recompute = rc
        ctx.recompute_y2 = rc >= 2 and not defer and not defer_skip   # those save y2 anyway
        ctx.b1 = b1 if rc else None
        ctx.b2 = b2 if ctx.recompute_y2 else None
        empty = torch.empty(0, device=y1.device, dtype=y1.dtype)
        y1_keep = empty if rc else y1
        y2_keep = empty if ctx.recompute_y2 else y2
        if defer:
            # deferred activation: the block hands out its PRE-BN output y2 with the BN
            # statistics s2; the consumer (transposed conv / head kernels) applies BN + ReLU
            # on load and returns dL/da2 with BN-backward partial sums attached
            ctx.has_x2 = x2 is not None
            ctx.x1_requires_grad = ctx.needs_input_grad[0]
            ctx.save_for_backward(x1, x2 if x2 is not None else torch.empty(0), y1_keep, y2, s1,
                                  s2, g1, g2)                     # (y2: the output itself)
            ctx.set_materialize_grads(False)
            ctx.mark_non_differentiable(s2)
            return y2, None, s2
        if defer_skip:
            # the skip leaves as y2 (its BN + ReLU is applied by the decoder's concat conv);
            # only the pooled activation is written.  s2 rides along (non-differentiable)
            _, pooled = F.bn_relu_apply(y2, s2, True, False)
            ctx.has_x2 = x2 is not None
            ctx.x1_requires_grad = ctx.needs_input_grad[0]
            ctx.save_for_backward(x1, x2 if x2 is not None else torch.empty(0), y1_keep, y2, s1,
                                  s2, g1, g2)
            ctx.set_materialize_grads(False)
            ctx.mark_non_differentiable(s2)
            return y2, pooled, s2
        a2, pooled = F.bn_relu_apply(y2, s2, pool)
        ctx.has_x2 = x2 is not None
        ctx.x1_requires_grad = ctx.needs_input_grad[0]
        ctx.save_for_backward(x1, x2 if x2 is not None else torch.empty(0), y1_keep, y2_keep, s1,
                              s2, g1, g2)
        ctx.set_materialize_grads(False)
        if pool:
            return a2, pooled, None
        return a2, None, None

    @staticmethod
    def _group_forward(ctx, x1, x2, b1, b2, g1, g2, blk, pool: bool, G: int, defer: bool = False):
        """A batched window of G micro-batches (``UNetEngine.bn_groups``): the convolutions
        run over the whole batch, every BatchNorm normalises each micro-batch with its own
        statistics (ref.py:580,583 at batch_size 1).

        Fused (``UNetEngine.group_fused``, the large levels): the convs walk their tiles
        group-major, so each conv's epilogue writes per-group BN statistic rows (no
        statistics pass), the second conv applies the per-group BN1 + ReLU in its prologue
        (a1 is never materialised) and its weight gradient re-applies it on load.
        Otherwise BN + ReLU is materialised per group (a1) and the convs read it plainly.
        a2 (+ pool) is materialised in both — except for the last decoder block with
        ``defer`` (``UNetEngine.group_head_defer``): it hands out the pre-BN y2 and the group
        statistics to the C = 32 head kernels, which apply each group's BN + ReLU on load and
        return the two-pass head gradient with group-major BN-backward partial rows.  y1 / y2
        stay for the backward."""
        F = _ops()
        p1, p2 = blk.pack1, blk.pack2
        fused = blk.engine.group_fused(x1, G, p1.cout)
        ctx.fused = fused
        if fused:
            count = float(x1.shape[0] // G * x1.shape[1] * x1.shape[2])   # pixels per group
            y1, _, r1 = F.conv3_fwd(x1, x2, p1.fwd, b1, None, None, p1.cout, 0, True,
                                    None, None, None, None, G)
            s1 = blk.bn1.finalize_group_rows(r1, G, count)
            y2, _, r2 = F.conv3_fwd(y1, None, p2.fwd, b2, s1[:, 2], s1[:, 3], p2.cout, 0, True,
                                    None, None, None, None, G)
            s2 = blk.bn2.finalize_group_rows(r2, G, count)
            a1 = torch.empty(0, device=y1.device, dtype=y1.dtype)
        else:
            y1 = F.conv3_fwd(x1, x2, p1.fwd, b1, None, None, p1.cout, 0, False)[0]
            s1 = blk.bn1.finalize_groups(y1, G)
            a1 = F.bn_group_apply(y1, s1, G, False)[0]
            y2 = F.conv3_fwd(a1, None, p2.fwd, b2, None, None, p2.cout, 0, False)[0]
            s2 = blk.bn2.finalize_groups(y2, G)
        ctx.groups = G
        ctx.blk, ctx.pool, ctx.defer = blk, pool, defer
        ctx.has_x2 = x2 is not None
        if defer:
            assert not pool, "BN groups: only the head's input is deferred"
            ctx.save_for_backward(x1, x2 if x2 is not None else torch.empty(0), y1, y2, s1, s2, g1,
                                  g2, a1)
            ctx.set_materialize_grads(False)
            ctx.mark_non_differentiable(s2)
            return y2, None, s2
        a2, pooled = F.bn_group_apply(y2, s2, G, pool)
        ctx.save_for_backward(x1, x2 if x2 is not None else torch.empty(0), y1, y2, s1, s2, g1,
                              g2, a1)
        ctx.set_materialize_grads(False)
        return a2, (pooled if pool else None), None

    @staticmethod
    def _group_backward(ctx, da2, dpool):
        F = _ops()
        x1, x2, y1, y2, s1, s2, g1, g2, a1 = ctx.saved_tensors
        blk = ctx.blk
        eng = blk.engine
        G = ctx.groups
        x2 = x2 if ctx.has_x2 else None
        if da2 is None and dpool is None:
            return (None,) * 15
        if da2 is not None and not ctx.defer:
            da2 = da2.contiguous()
        dpool = dpool.contiguous() if dpool is not None else None
        bn1, bn2 = blk.bn1.bn, blk.bn2.bn
        p1, p2 = blk.pack1, blk.pack2
        w1 = blk.conv1.weight
        direct = eng.direct_grads
        fused = ctx.fused
        # (fused: conv2's input is relu(bn1(y1)) per group, formed on load from y1)
        xw2, psc, psh = (y1, s1[:, 2], s1[:, 3]) if fused else (a1, None, None)
        # deferred into the head: its second pass recomputes dA and applies each group's BN2
        # backward (group-major partial rows from the fused forward, at unit scale)
        head = getattr(da2, "_ddlpc_head", None) if (ctx.defer and da2 is not None) else None
        if ctx.defer and head is None:
            raise RuntimeError("BN groups: the deferred head input has a second autograd consumer")
        hargs = ((*head, s2, da2._ddlpc_bn_partial, g2) if head is not None else None)
        hps = getattr(da2, "_ddlpc_bn_pscale", None) if head is not None else None
        # ---- second conv: per-group BN2 + ReLU (+ unpool + skip sum) backward
        if head is not None:
            dy2, dg2, dbe2 = F.head_ce_bn_bwd(*hargs, bn2.weight.grad if direct else None,
                                              bn2.bias.grad if direct else None, hps, G)
        else:
            dy2, dg2, dbe2 = F.bn_group_backward(da2, dpool, y2, s2, g2, G,
                                                 bn2.weight.grad if direct else None,
                                                 bn2.bias.grad if direct else None)
        if direct:
            dg2 = dbe2 = None
        # its gradients: at 32 -> 32 channels on the fused levels one kernel (conv3x3_bwd32,
        # group-major) for both; otherwise the weight gradient (per-group prologue when fused)
        # and the data gradient (per-group BN1-backward partials in its epilogue when fused)
        g32 = fused and eng.bwd32 and p2.cin == 32 and p2.cout == 32
        part1 = None
        dw2 = None
        if g32:
            if direct:
                da1, part1, _ = F.conv3_bwd32(dy2, y1, s1, p2.dgrad, blk.conv2.weight.grad, G)
                with eng.wgrad_stream():
                    eng.ready(bn2.weight, bn2.bias, blk.conv2.weight, blk.conv2.bias)
            else:
                da1, part1, dw2 = F.conv3_bwd32(dy2, y1, s1, p2.dgrad, None, G)
                dw2 = dw2.view_as(blk.conv2.weight)
        else:
            if direct:
                with eng.wgrad_stream(dy2, xw2, s1):
                    F.conv3_wgrad(dy2, xw2, None, psc, psh, blk.conv2.weight.grad, groups=G)
                    eng.ready(bn2.weight, bn2.bias, blk.conv2.weight, blk.conv2.bias)
            else:
                dw2 = F.conv3_wgrad(dy2, xw2, None, psc, psh, groups=G).view_as(blk.conv2.weight)
            if fused:
                da1, _, part1 = F.conv3_fwd(dy2, None, p2.dgrad, None, None, None, p2.cin, 0, False,
                                            None, None, y1, s1, G)
            else:
                da1 = F.conv3_fwd(dy2, None, p2.dgrad, None, None, None, p2.cin, 0, False)[0]
        # ---- first conv
        padded_in = x2 is None and x1.shape[-1] != w1.shape[1]     # first layer: 3 -> 8 ch
        if direct:
            dy1 = F.bn_group_backward(da1, None, y1, s1, g1, G, bn1.weight.grad, bn1.bias.grad,
                                      part1)[0]
            with eng.wgrad_stream(dy1, x1, x2):
                if padded_in:
                    w1.grad.add_(F.conv3_wgrad(dy1, x1, None, None, None,
                                               cin_real=w1.shape[1])[:, :w1.shape[1]])
                else:
                    F.conv3_wgrad(dy1, x1, x2, None, None, w1.grad)
                eng.ready(bn1.weight, bn1.bias, w1, blk.conv1.bias)
            dg1 = dbe1 = dw1 = None
        else:
            dy1, dg1, dbe1 = F.bn_group_backward(da1, None, y1, s1, g1, G, None, None, part1)
            dw1 = F.conv3_wgrad(dy1, x1, x2, None, None, None,
                                cin_real=w1.shape[1] if padded_in else 0)
            dw1 = (dw1[:, :w1.shape[1]] if padded_in else dw1).reshape(w1.shape)
        dx1 = dx2 = None
        if ctx.needs_input_grad[0] or (x2 is not None and ctx.needs_input_grad[1]):
            co1 = x1.shape[-1] if x2 is not None else 0
            want_sums = x2 is not None and blk.up_is_convt
            dx1, dx2, sums = F.conv3_fwd(dy1, None, p1.dgrad, None, None, None, p1.cin, co1,
                                         want_sums)
            if want_sums:
                dx1._ddlpc_colsum_rows = sums
            if x2 is None:
                dx2 = None
        if blk.first:
            eng.join()
        zb1 = torch.zeros_like(g1) if (not direct and ctx.needs_input_grad[3]) else None
        zb2 = torch.zeros_like(g2) if (not direct and ctx.needs_input_grad[7]) else None
        return (dx1, dx2, dw1, zb1, dg1, dbe1, dw2, zb2, dg2, dbe2, None, None, None, None, None)

    @staticmethod
    def backward(ctx, da2, dpool, _ds2):
        if ctx.groups:
            return _DoubleConvFn._group_backward(ctx, da2, dpool)
        F = _ops()
        x1, x2, y1, y2, s1, s2, g1, g2 = ctx.saved_tensors
        blk = ctx.blk
        eng = blk.engine
        x2 = x2 if ctx.has_x2 else None
        # head gradient still to be formed (two-pass head backward, see _HeadCEFn)
        head = getattr(da2, "_ddlpc_head", None) if (ctx.defer and da2 is not None) else None
        if (ctx.defer and head is None and da2 is not None and da2.dim() > 0
                and all(st == 0 for st in da2.stride())):
            # the head's zero-stride stand-in lost its attribute: another autograd consumer
            # of the deferred output summed into it, so the head's gradient would be dropped
            raise RuntimeError("deferred block output has a second autograd consumer besides "
                               "the two-pass head; set engine.head_apply = False")
        if da2 is not None and head is None:
            da2 = da2.contiguous()
        if dpool is not None:
            dpool = dpool.contiguous()
        if da2 is None and dpool is None:
            return (None,) * 15
        x2_bn = ctx.x2_bn
        sc2 = x2_bn[2] if x2_bn is not None else None
        sh2 = x2_bn[3] if x2_bn is not None else None
        if ctx.recompute:
            y1 = F.conv3_fwd(x1, x2, blk.pack1.fwd, ctx.b1, None, None, blk.pack1.cout, 0, False,
                             sc2, sh2)[0]
        if ctx.recompute_y2:
            y2 = F.conv3_fwd(y1, None, blk.pack2.fwd, ctx.b2, s1[2], s1[3], blk.pack2.cout, 0, False)[0]
        # BN-backward partial sums already reduced by the consumer's kernel (deferred BN)
        part2 = getattr(da2, "_ddlpc_bn_partial", None) if ctx.defer else None
        bn1, bn2 = blk.bn1.bn, blk.bn2.bn
        direct = eng.direct_grads
        p1, p2 = blk.pack1, blk.pack2
        # the 32-channel level: conv2's data and weight gradients in ONE kernel that reads dY2
        # and y1 once (conv3x3_bwd32.hip; BN1-backward partials in its epilogue)
        bwd32 = (eng.bwd32 and eng.bnb_epilogue and y1.dim() == 4 and p2.cin == 32 and
                 p2.cout == 32)
        # ---- second conv: BN2 + ReLU (+ unpool + skip sum) backward, then its gradients
        if direct:
            if head is not None:
                dy2, _, _ = F.head_ce_bn_bwd(*head, s2, part2, g2, bn2.weight.grad, bn2.bias.grad,
                                             getattr(da2, "_ddlpc_bn_pscale", None))
            else:
                dy2, _, _ = F.bn_backward(da2, dpool, y2, s2, g2, None, bn2.weight.grad,
                                          bn2.bias.grad, part2)
            if bwd32:
                da1, part1, _ = F.conv3_bwd32(dy2, y1, s1, p2.dgrad, blk.conv2.weight.grad)
                with eng.wgrad_stream():
                    eng.ready(bn2.weight, bn2.bias, blk.conv2.weight, blk.conv2.bias)
            else:
                with eng.wgrad_stream(dy2, y1, s1):
                    F.conv3_wgrad(dy2, y1, None, s1[2], s1[3], blk.conv2.weight.grad)
                    eng.ready(bn2.weight, bn2.bias, blk.conv2.weight, blk.conv2.bias)
            dg2 = dbe2 = dw2 = None
        else:
            if head is not None:
                dy2, dg2, dbe2 = F.head_ce_bn_bwd(*head, s2, part2, g2, None, None,
                                                  getattr(da2, "_ddlpc_bn_pscale", None))
            else:
                dy2, dg2, dbe2 = F.bn_backward(da2, dpool, y2, s2, g2, None, None, None, part2)
            if bwd32:
                da1, part1, dw2 = F.conv3_bwd32(dy2, y1, s1, p2.dgrad)
                dw2 = dw2.view_as(blk.conv2.weight)
            else:
                dw2 = F.conv3_wgrad(dy2, y1, None, s1[2], s1[3]).view_as(blk.conv2.weight)
        if not bwd32 and eng.bnb_epilogue and y1.dim() == 4:
            # the epilogue also reduces BN1 backward's (sum dyh, sum dyh*xhat) against y1
            da1, _, part1 = F.conv3_fwd(dy2, None, p2.dgrad, None, None, None, p2.cin, 0, False,
                                        None, None, y1, s1)
        elif not bwd32:
            part1 = None
            da1, _, _ = F.conv3_fwd(dy2, None, p2.dgrad, None, None, None, p2.cin, 0, False)
        # ---- first conv
        w1 = blk.conv1.weight
        padded_in = x2 is None and x1.shape[-1] != w1.shape[1]   # first layer: 3 -> 8 ch
        # first block, input gradient not wanted: the weight gradient is BN1 backward's only
        # consumer, so it applies that backward on load (dY prologue) from dA1 and y1 — the
        # apply pass (read dA1 + y1, write dY1) is skipped
        wg_pro = (padded_in and part1 is not None and eng.wgrad_dy_prologue and
                  not ctx.needs_input_grad[0])
        # 32-output-channel concat conv (dec1.a): its weight-gradient kernel (every input
        # chunk per workgroup) applies BN1's backward on load from dA1 and y1 and stores the
        # formed dY1 for the data gradient — no separate apply pass (read dA1 + y1, write dY1).
        # It runs on the compute stream: the data gradient below reads its dY1
        c32p = (not wg_pro and part1 is not None and eng.c32_bnp and x2_bn is None and
                eng.c32_eligible(x1, x2, w1.shape[0]))
        if c32p:
            dy1 = torch.empty_like(da1)
            if direct:
                coefs, _, _ = F.bn_grad_coefs(part1, y1, s1, g1, bn1.weight.grad, bn1.bias.grad)
                F.conv3_wgrad(da1, x1, x2, None, None, w1.grad, None, None, y1, s1, coefs,
                              dy_out=dy1)
                with eng.wgrad_stream():     # (readiness after both streams' writes)
                    eng.ready(bn1.weight, bn1.bias, w1, blk.conv1.bias)
                dg1 = dbe1 = dw1 = None
            else:
                coefs, dg1, dbe1 = F.bn_grad_coefs(part1, y1, s1, g1)
                dw1 = F.conv3_wgrad(da1, x1, x2, None, None, None, None, None, y1, s1, coefs,
                                    dy_out=dy1).reshape(w1.shape)
        elif direct and wg_pro:
            coefs, _, _ = F.bn_grad_coefs(part1, y1, s1, g1, bn1.weight.grad, bn1.bias.grad)
            with eng.wgrad_stream(da1, y1, x1, coefs, s1):
                w1.grad.add_(F.conv3_wgrad(da1, x1, None, None, None, None, None, None,
                                           y1, s1, coefs, cin_real=w1.shape[1])[:, :w1.shape[1]])
                eng.ready(bn1.weight, bn1.bias, w1, blk.conv1.bias)
            dg1 = dbe1 = dw1 = None
        elif wg_pro:
            coefs, dg1, dbe1 = F.bn_grad_coefs(part1, y1, s1, g1)
            dw1 = F.conv3_wgrad(da1, x1, None, None, None, None, None, None, y1, s1, coefs,
                                cin_real=w1.shape[1])
            dw1 = dw1[:, :w1.shape[1]].reshape(w1.shape)
        elif direct:
            dy1, _, _ = F.bn_backward(da1, None, y1, s1, g1, None, bn1.weight.grad, bn1.bias.grad,
                                      part1)
            with eng.wgrad_stream(dy1, x1, x2, x2_bn):
                if padded_in:
                    w1.grad.add_(F.conv3_wgrad(dy1, x1, None, None, None,
                                               cin_real=w1.shape[1])[:, :w1.shape[1]])
                else:
                    F.conv3_wgrad(dy1, x1, x2, None, None, w1.grad, sc2, sh2)
                eng.ready(bn1.weight, bn1.bias, w1, blk.conv1.bias)
            dg1 = dbe1 = dw1 = None
        else:
            dy1, dg1, dbe1 = F.bn_backward(da1, None, y1, s1, g1, None, None, None, part1)
            dw1 = F.conv3_wgrad(dy1, x1, x2, None, None, None, sc2, sh2,
                                cin_real=w1.shape[1] if padded_in else 0)
            dw1 = (dw1[:, :w1.shape[1]] if padded_in else dw1).reshape(w1.shape)
        dx1 = dx2 = None
        if not wg_pro and (ctx.needs_input_grad[0] or (x2 is not None and ctx.needs_input_grad[1])):
            c_x1 = x1.shape[-1]
            co1 = c_x1 if x2 is not None else 0
            # for a decoder block dx1 is the transposed conv's output gradient: keep the
            # epilogue's per-channel sums, they are that conv's bias gradient
            want_sums = x2 is not None and blk.up_is_convt
            dx1, dx2, sums = F.conv3_fwd(dy1, None, p1.dgrad, None, None, None, p1.cin, co1,
                                         want_sums)
            if want_sums:
                dx1._ddlpc_colsum_rows = sums
            if x2 is None:
                dx2 = None
        if blk.first:
            eng.join()                   # last backward node: main stream waits for wgrads
        # conv biases feeding a training-mode BN have an exactly-zero gradient
        zb1 = torch.zeros_like(g1) if (not direct and ctx.needs_input_grad[3]) else None
        zb2 = torch.zeros_like(g2) if (not direct and ctx.needs_input_grad[7]) else None
        return (dx1, dx2, dw1, zb1, dg1, dbe1, dw2, zb2, dg2, dbe2, None, None, None, None, None)


class _ConvTFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pack: _ConvPack, engine, bn: Optional[torch.Tensor] = None):
        # bn: statistics of a deferred-BN input (x = pre-BN y2 of the previous block)
        out = _ops().convt_fwd(x, pack.fwd, b, pack.cout, bn)
        ctx.save_for_backward(x, bn if bn is not None else torch.empty(0))
        ctx.has_bn = bn is not None
        ctx.pack = pack
        ctx.engine = engine
        return out

    @staticmethod
    def backward(ctx, dout):
        F = _ops()
        x, bn = ctx.saved_tensors
        bn = bn if ctx.has_bn else None
        dout = dout.contiguous()
        eng = ctx.engine
        conv = ctx.pack.conv
        rows = getattr(dout, "_ddlpc_colsum_rows", None)
        if (eng.convt_fused and ctx.needs_input_grad[0] and x.dim() == 4 and x.shape[-1] == 64
                and ctx.pack.cout == 64):
            # 64 -> 64-channel 2-D transposed conv (the 256^2 level): one kernel reads dOut
            # once for both gradients (convt_bwd_fused; other shapes fall back inside)
            if eng.direct_grads:
                dx, part, _, _ = F.convt_bwd_fused(x, dout, ctx.pack.dgrad, conv.weight.grad,
                                                   conv.bias.grad, rows, bn)
                with eng.wgrad_stream():
                    eng.ready(conv.weight, conv.bias)
                dw = db = None
            else:
                dx, part, dw, db = F.convt_bwd_fused(x, dout, ctx.pack.dgrad, None, None, rows, bn)
                dw = dw.view_as(conv.weight)
            if bn is not None:
                dx._ddlpc_bn_partial = part
            return dx, dw, db, None, None, None
        dx = None
        if ctx.needs_input_grad[0]:
            dx, part = F.convt_dgrad(dout, ctx.pack.dgrad, ctx.pack.cin, x if bn is not None else None,
                                     bn)
            if bn is not None:
                dx._ddlpc_bn_partial = part
        if eng.direct_grads:
            if eng.side_convt:
                with eng.wgrad_stream(x, dout, rows, bn):
                    F.convt_wgrad(x, dout, conv.weight.grad, conv.bias.grad, rows, bn)
                    eng.ready(conv.weight, conv.bias)
            else:
                F.convt_wgrad(x, dout, conv.weight.grad, conv.bias.grad, rows, bn)
                with eng.wgrad_stream():
                    eng.ready(conv.weight, conv.bias)
            return dx, None, None, None, None, None
        dw, db = F.convt_wgrad(x, dout, None, None, rows, bn)
        return dx, dw.view_as(conv.weight), db, None, None, None


class _BilinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _ops().bilinear_up2(x)

    @staticmethod
    def backward(ctx, dy):
        return _ops().bilinear_up2_bwd(dy.contiguous())


class _HeadCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, wh, bh, labels, ignore_index: int, engine,
                bn: Optional[torch.Tensor] = None):
        # training with the deferred BN: the forward also runs the backward's statistics
        # pass (unit gradient scale) — one read of the activation and labels for both
        ctx.rows = None
        # (Function.forward runs with grad mode off: needs_input_grad says whether a
        # backward will follow)
        # (BN groups: bn = [groups][4][C] per-group statistics, fused forward only —
        # UNetEngine.group_head_defer)
        groups = bn.shape[0] if (bn is not None and bn.dim() == 3) else 0
        if (bn is not None and engine.head_apply and engine.head_fused_fwd
                and any(ctx.needs_input_grad[:3])):
            out3, wrows, brows = _ops().head_ce_fwd_stats(a, wh, bh, labels, ignore_index, bn, groups)
            ctx.rows = (wrows, brows)
        else:
            assert groups == 0, "grouped head statistics need the fused training forward"
            out3 = _ops().head_ce_fwd(a, wh, bh, labels, ignore_index, bn)
        ctx.save_for_backward(a, wh, bh, labels, out3, bn if bn is not None else torch.empty(0))
        ctx.has_bn = bn is not None
        ctx.ignore_index = ignore_index
        ctx.engine = engine
        loss = out3[0]
        correct = out3[1]
        ctx.mark_non_differentiable(correct)
        return loss, correct

    @staticmethod
    def backward(ctx, dloss, dcorrect):
        a, wh, bh, labels, out3, bn = ctx.saved_tensors
        bn = bn if ctx.has_bn else None
        gs = dloss.reshape(1).float().contiguous() if dloss is not None else None
        eng = ctx.engine
        # two-pass backward with the deferred BatchNorm: this pass reduces dWh, dbh and the
        # BN partials without storing dA; the block's backward then runs head_ce_bn_bwd,
        # which recomputes dA and applies the BatchNorm backward in registers (no dA
        # round trip through HBM, no separate BN-apply pass).  engine.head_apply = False: one pass
        two_pass = bn is not None and eng.head_apply
        if ctx.rows is not None:
            # statistics already reduced by the forward at unit scale: scale = dL / count
            wrows, brows = ctx.rows
            scale = _ops().head_grad_scale(out3, gs)       # one launch, on the device
            K, C = wh.shape
            head = eng.head
            if eng.direct_grads:
                _ops().head_wgrad_from_rows(wrows, scale, K, C, head.weight.grad, head.bias.grad)
                with eng.wgrad_stream():
                    eng.ready(head.weight, head.bias)
                dw = db = None
            else:
                dw, db = _ops().head_wgrad_from_rows(wrows, scale, K, C)
            da = eng.zero_scalar(a).expand(a.shape)
            da._ddlpc_head = (a, wh, bh, labels, out3, gs, ctx.ignore_index)
            da._ddlpc_bn_partial = brows
            da._ddlpc_bn_pscale = scale
            return da, dw, db, None, None, None, None
        if eng.direct_grads:
            head = eng.head
            da, _, _, part = _ops().head_ce_bwd(a, wh, bh, labels, out3, gs, ctx.ignore_index,
                                                head.weight.grad, head.bias.grad, bn, not two_pass)
            with eng.wgrad_stream():
                eng.ready(head.weight, head.bias)
            dw = db = None
        else:
            da, dw, db, part = _ops().head_ce_bwd(a, wh, bh, labels, out3, gs, ctx.ignore_index,
                                                  None, None, bn, not two_pass)
        if two_pass:
            # stand-in gradient of the right shape (no storage); the consumer recognises it
            da = eng.zero_scalar(a).expand(a.shape)
            da._ddlpc_head = (a, wh, bh, labels, out3, gs, ctx.ignore_index)
        if bn is not None:
            da._ddlpc_bn_partial = part
        return da, dw, db, None, None, None, None


class _Block:
    """Kernel-side view of one DoubleConv: packed weights + BN handles."""

    def __init__(self, dc: nn.Module, first: bool, engine, up_is_convt: bool = False):
        self.engine = engine
        self.up_is_convt = up_is_convt
        self.first = first
        seq = dc.double_conv
        self.conv1, self.conv2 = seq[0], seq[3]
        self.bn1, self.bn2 = _BNState(seq[1], engine), _BNState(seq[4], engine)
        self.pack1 = _ConvPack(self.conv1, 0, need_dgrad=not first)
        self.pack2 = _ConvPack(self.conv2, 0, need_dgrad=True)

    def __call__(self, x1, x2, pool: bool, defer: bool = False, x2_bn=None, defer_skip=False):
        """-> (activation, pooled | None, None) or, deferred, (pre-BN y2, None, stats s2), or
        with defer_skip (pre-BN y2 as the skip, pooled, stats s2)."""
        return _DoubleConvFn.apply(x1, x2, self.conv1.weight, self.conv1.bias,
                                   self.bn1.bn.weight, self.bn1.bn.bias, self.conv2.weight,
                                   self.conv2.bias, self.bn2.bn.weight, self.bn2.bn.bias, self,
                                   pool, defer, x2_bn, defer_skip)


def check_supported(model: nn.Module):
    """Fail loudly on geometries the kernels do not tile (instead of a mid-step TORCH_CHECK):
    every conv width a multiple of 8 (16-byte channel-last pixels), the up-sampled half of
    each concat and every transposed conv a multiple of 32 channels, a head over 8/16/32/64
    channels and at most 16 classes."""
    w = list(model.enc_widths)
    k = model.conv_last.weight.shape[0]
    problems = []
    if any(c % 8 for c in w):
        problems.append(f"widths {w} must be multiples of 8")
    if any(c % 32 for c in w[1:]):
        problems.append(f"decoder concat / transposed-conv widths {w[1:]} must be multiples of 32")
    if w[0] not in (8, 16, 32, 64):
        problems.append(f"head input width {w[0]} not in (8, 16, 32, 64)")
    if not 1 <= k <= 16:
        problems.append(f"out_classes {k} not in [1, 16]")
    if problems:
        raise ValueError("HIP engine: unsupported U-Net geometry: " + "; ".join(problems) +
                         " (use impl='torch' for this configuration)")


def bn_groups_supported(model: nn.Module, tile: int) -> bool:
    """Whether every BatchNorm of a ``models.UNet`` fits the per-micro-batch group kernels
    (``csrc/bn.hip`` bn_group_supported): C a multiple of 8 with C / 8 a power of two
    <= 256, and even spatial extents at the pooled (encoder) BatchNorms."""
    def ok(c: int) -> bool:
        g = c // 8
        return c % 8 == 0 and 0 < g <= 256 and (g & (g - 1)) == 0
    bns = [m for m in model.modules() if isinstance(m, (nn.BatchNorm2d, nn.BatchNorm3d))]
    if not all(ok(b.num_features) for b in bns):
        return False
    return all((tile >> lvl) >= 2 and (tile >> lvl) % 2 == 0
               for lvl in range(len(list(model.down_blocks()))))


class _SideSegment:
    """``with`` body runs on the engine's side stream; on exit an event marks the segment's
    end for the lag bound (``UNetEngine.wgrad_stream``)."""

    def __init__(self, eng, cur, nbytes):
        self.eng, self.cur, self.nbytes = eng, cur, nbytes
        self.ctx = torch.cuda.stream(eng.side)

    def __enter__(self):
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        ev = torch.cuda.Event()
        ev.record(self.eng.side)
        r = self.ctx.__exit__(*exc)
        self.eng._retire(self.cur, ev, self.nbytes)
        return r


class UNetEngine:
    """Runs a ``models.UNet`` through the ``torch.ops.ddlpc`` operators (attach with
    ``UNet.to_hip()``): the gfx950 kernels for a model on the GPU, the C++ reference kernels
    (csrc/cpu_ref.cpp) for a model on the CPU — one code path, device dispatch by PyTorch.
    The side stream for weight gradients exists on the GPU only."""

    def __init__(self, model: nn.Module, strict: bool = True):
        _ext.load(strict=strict)
        check_supported(model)
        self.model = model
        dev = next(model.parameters()).device
        # (any device: torch.ops.ddlpc dispatches to the gfx950 kernels for GPU tensors and
        # to the C++ reference kernels of csrc/cpu_ref.cpp for CPU tensors)
        cuda = dev.type == "cuda"
        # direct_grads: kernels accumulate straight into the (flat) .grad buffers and report
        # readiness through ``grad_ready`` (the DP reducer's bucket trigger) instead of
        # returning gradients for autograd to add.  Enabled by the Trainer once parameters
        # are flattened.
        self.direct_grads = False
        self.grad_ready = None
        # weight gradients (3x3 wgrad + its split-K reduction, convT wgrad) run on a side
        # HIP stream, concurrently with the data-gradient chain on the compute stream: the
        # two chains are independent until the optimizer step, and the small deep-layer
        # kernels of one fill the CUs the other leaves idle.  DDLPC_WGRAD_STREAM=0 disables.
        use_side = os.environ.get("DDLPC_WGRAD_STREAM", "1") != "0"
        # (stream priorities measured within +-0.3%: a plain stream,
        # profiles/r5/rows_sum_4wave_g66/)
        self.side = torch.cuda.Stream(dev) if (use_side and cuda) else None
        self._side_stream = self.side
        self._side_used = False
        # memory the side stream's lag may hold back (see ``wgrad_stream``): default 6% of
        # HBM (17 GB on MI355X; measured at 1024^2 x 128: 43 GB still ran out of HBM, 16 GB
        # did not; 256^2 x 128 never reaches it), DDLPC_SIDE_LAG_GB overrides
        lag_gb = os.environ.get("DDLPC_SIDE_LAG_GB")
        self.side_lag_bytes = (int(float(lag_gb) * 2**30) if lag_gb else
                               int(0.06 * torch.cuda.get_device_properties(dev).total_memory)
                               if cuda else 0)
        self._lag: List[Tuple[torch.cuda.Event, int]] = []
        self._lag_bytes = 0
        self.lag_waits = 0
        # deferred BatchNorm activations (see ``features``): "all" | "convt" | "none"
        self.defer_mode = "all"
        # transposed-conv weight gradients on the side stream too
        self.side_convt = True
        self.recompute = 0               # Trainer sets cfg.recompute: 0 / 1 (y1) / 2 (y1, y2)
        # per-micro-batch BatchNorm groups of a batched accumulation window (Trainer
        # bn_window): G >= 1 = the training batch is G micro-batches, each normalised with
        # its own statistics (no deferred BN / prologue fusion in this mode; G = 1 runs one
        # micro-batch through the same unfused kernels); 0 = the fused path
        self.bn_groups = 0
        # BN groups: fuse the statistics / BN1 prologue / BN1-backward reduction into the
        # convs (group-major tiles, ``_DoubleConvFn._group_forward``) on levels with at least
        # this many pixels per group: smaller levels have too few tiles per group to keep
        # every CU busy (and their unfused passes are cheap); None disables
        self.group_fuse_min_px: Optional[int] = 16384
        # encoder skips handed out pre-BN (see ``defer_skip_levels``): saves ~1 GB at
        # 256^2 x 128 but measured ~1.2% slower end to end (docs/PERF.md), so opt-in
        # (tests/test_unet_gpu.py::test_deferred_skips_match_materialised_engine runs both)
        self.defer_skip = False
        self.defer_skip_max_level = 99          # (with defer_skip: only levels <= this one)
        # BN1 backward's reduction pass fused into the epilogue of the data gradient that
        # produces its input gradient (2-D; False: separate reduction kernel)
        self.bnb_epilogue = True
        # two-pass head backward with the last block's BN backward fused into the second
        # pass (see _HeadCEFn.backward; False: dA stored + separate BN apply)
        self.head_apply = True
        # ... and its statistics pass fused into the training forward (False: separate
        # forward and statistics passes)
        self.head_fused_fwd = True
        # 64 -> 64-channel transposed conv: data + weight gradient in one kernel
        # (False: separate kernels, weight gradient on the side stream)
        self.convt_fused = True
        # first block: BN1 backward applied on load by its weight gradient (no apply pass;
        # False: separate bn_backward)
        self.wgrad_dy_prologue = True
        # 32 -> 32-channel second convs: data + weight gradient in one kernel (conv3x3_bwd32;
        # False: the resident data gradient + the v3 weight gradient on the side stream)
        self.bwd32 = True
        # 32-output-channel concat convs (dec1.a): BN1 backward applied on load by the weight
        # gradient, which stores dY1 for the data gradient (False: separate apply pass)
        self.c32_bnp = True
        self.enc = [_Block(b.double_conv, first=(i == 0), engine=self)
                    for i, b in enumerate(model.down_blocks())]
        self.mid = _Block(model.double_conv, first=False, engine=self)
        self.dec = []
        for ub in model.up_blocks():
            up = ub.up_sample
            pack = _ConvPack(up, 1, True) if isinstance(up, (nn.ConvTranspose2d, nn.ConvTranspose3d)) else None
            self.dec.append((ub, pack, _Block(ub.double_conv, first=False, engine=self,
                                              up_is_convt=pack is not None)))
        head = model.conv_last
        self.head = head
        # deferred BatchNorm running statistics (concurrent micro-batch streams, Trainer
        # micro_streams): bn_defer_j = the stream whose slot vector the forward being queued
        # writes (None: update the running statistics in place)
        self.bns = [b for blk in self.enc + [self.mid] + [d[2] for d in self.dec]
                    for b in (blk.bn1, blk.bn2)]
        for i, b in enumerate(self.bns):
            b.index = i
        self.bn_defer_j: Optional[int] = None
        self._zeros = {}
        self._bn_streams: List[torch.Tensor] = []
        self._bn_views: List[List[torch.Tensor]] = []
        self._bn_offs: List[int] = []
        self._bn_arena: Optional[torch.Tensor] = None
        self.packs = [p for b in self.enc + [self.mid] for p in (b.pack1, b.pack2)]
        for _, pk, b in self.dec:
            self.packs += [pk, b.pack1, b.pack2] if pk is not None else [b.pack1, b.pack2]
        self._entries = None
        self._entries_key = None
        self._version = None
        self.pack_weights()

    def zero_scalar(self, like: torch.Tensor) -> torch.Tensor:
        """A cached 0-d zero of ``like``'s dtype/device (base of the head's zero-stride
        stand-in gradient: no fill kernel per step)."""
        key = (like.dtype, like.device)
        z = self._zeros.get(key)
        if z is None:
            z = self._zeros[key] = torch.zeros((), dtype=like.dtype, device=like.device)
        return z

    # ------------------------------------------------------------------ deferred BN stats
    def bn_defer_prepare(self, K: int, n: int):
        """Storage for deferred BatchNorm running statistics: per stream k (K concurrent
        micro-batch streams) one flat slot vector [sum over BN layers of 2C] written by the
        forwards queued on that stream (bn_finalize with momentum 1 writes (mean, unbiased
        var) exactly), and an arena [n][same] that receives stream k's vector after each of
        its micro-batches (``bn_defer_stash``).  Slots are zeroed once and then only ever
        hold finite values (the momentum-1 update reads them as 0 * old)."""
        total = sum(2 * b.bn.num_features for b in self.bns)
        dev = self.bns[0].bn.running_mean.device
        if len(self._bn_streams) < K:
            self._bn_offs, o = [], 0
            for b in self.bns:
                self._bn_offs.append(o)
                o += 2 * b.bn.num_features
            self._bn_streams = [torch.zeros(total, dtype=torch.float32, device=dev) for _ in range(K)]
            self._bn_views = [[v[o:o + 2 * b.bn.num_features].view(2, b.bn.num_features)
                               for o, b in zip(self._bn_offs, self.bns)] for v in self._bn_streams]
        if self._bn_arena is None or self._bn_arena.shape[0] < n:
            self._bn_arena = torch.zeros(n, total, dtype=torch.float32, device=dev)

    def bn_defer_slot(self, index: int, k: int) -> torch.Tensor:
        return self._bn_views[k][index]

    def bn_defer_stash(self, k: int, j: int):
        """Micro-batch j (queued on stream k, current stream): its slot vector -> arena row j."""
        self._bn_arena[j].copy_(self._bn_streams[k])

    def bn_defer_apply(self, n: int):
        """Apply the n deferred running-statistics updates of every BatchNorm in micro-batch
        order (one launch for the whole network when the BatchNorms share a momentum, else
        one per BatchNorm): bit-identical to n sequential forwards."""
        moms = {(b.bn.momentum if b.bn.momentum is not None else 0.1) for b in self.bns}
        if len(moms) == 1 and all(b.bn.track_running_stats for b in self.bns):
            key = (self._bn_arena.data_ptr(), tuple(b.bn.running_mean.data_ptr() for b in self.bns))
            if getattr(self, "_bn_all_key", None) != key:
                rows = [[b.bn.running_mean.data_ptr(), b.bn.running_var.data_ptr(),
                         b.bn.num_batches_tracked.data_ptr(),
                         b.bn.num_features | (off << 32)] for b, off in zip(self.bns, self._bn_offs)]
                self._bn_all = torch.tensor(rows, dtype=torch.int64).to(self._bn_arena.device)
                self._bn_all_key = key
                self._bn_all_maxc = max(b.bn.num_features for b in self.bns)
            _ops().bn_running_apply_all(self._bn_all, self._bn_arena, n, self._bn_all_maxc,
                                        float(moms.pop()))
            return
        for b, off in zip(self.bns, self._bn_offs):
            bn = b.bn
            if not bn.track_running_stats:
                continue
            mom = bn.momentum if bn.momentum is not None else 0.1
            c2 = 2 * bn.num_features
            _ops().bn_running_apply(bn.running_mean, bn.running_var,
                                    self._bn_arena[:n, off:off + c2], float(mom),
                                    bn.num_batches_tracked)

    def enable_direct_grads(self, grad_ready=None):
        for p in self.model.parameters():
            if p.grad is None or not p.grad.is_contiguous():
                raise RuntimeError("direct grads need persistent contiguous .grad buffers")
        self.direct_grads = True
        self.grad_ready = grad_ready

    def set_side_stream(self, enabled: bool):
        """Switch the weight-gradient side stream on/off between steps (see
        ``Trainer.choose_schedule``)."""
        dev = next(self.model.parameters()).device
        if enabled and self._side_stream is None and dev.type == "cuda":
            self._side_stream = torch.cuda.Stream(dev)
        self.join()
        self.side = self._side_stream if enabled else None

    def wgrad_stream(self, *tensors):
        """Context for weight-gradient work: the side stream first waits for everything
        queued so far on the compute stream; tensors allocated there and read on the side
        stream are marked so the caching allocator does not recycle them early.

        Lag bound: a freed tensor that was marked is only reusable once the side stream has
        run everything queued at the time of the free, so the memory held back grows with
        the side stream's lag.  At 1024^2 x batch 128 (169 GB resident) an unbounded lag
        ran the allocator out of HBM (free-and-retry, 3-6x slower steps: the "two-stream"
        slowdown at large batch).  When the marked
        bytes of the not-yet-retired side segments exceed ``side_lag_bytes`` the compute
        stream waits for the oldest ones (GPU-side event wait; the host never blocks)."""
        if self.side is None or not self.direct_grads or torch.cuda.is_current_stream_capturing():
            # (hipGraph replay runs the captured streams serially: no gain from forking)
            return contextlib.nullcontext()
        cur = torch.cuda.current_stream(self.side.device)
        self.side.wait_stream(cur)
        # (inside a hipGraph capture the allocator defers reuse of such blocks to the end
        # of the capture, so the replayed graph cannot race on them either)
        nbytes = 0
        for t in tensors:
            if isinstance(t, torch.Tensor) and t.numel() and t.is_cuda:
                t.record_stream(self.side)
                nbytes += t.numel() * t.element_size()
        self._side_used = True
        return _SideSegment(self, cur, nbytes)

    def join(self):
        """Compute stream waits for all queued weight-gradient work."""
        if self.side is not None and self._side_used:
            torch.cuda.current_stream(self.side.device).wait_stream(self.side)
            self._side_used = False
        self._lag, self._lag_bytes = [], 0

    def _retire(self, cur, ev, nbytes):
        self._lag.append((ev, nbytes))
        self._lag_bytes += nbytes
        while self._lag_bytes > self.side_lag_bytes and len(self._lag) > 1:
            ev0, nb0 = self._lag.pop(0)
            cur.wait_event(ev0)
            self._lag_bytes -= nb0
            self.lag_waits += 1

    def ready(self, *params):
        """Gradients of ``params`` are complete once the queued work finishes.  Called on
        the side stream (after it joined the compute stream), so a bucket collective the
        reducer launches here is ordered after every gradient write of either stream."""
        if self.grad_ready is not None:
            for p in params:
                self.grad_ready(p)

    # ------------------------------------------------------------------ weights
    def _params_version(self):
        return sum(p.conv.weight._version for p in self.packs)

    def pack_weights(self):
        key = tuple(p.conv.weight.data_ptr() for p in self.packs)
        if self._entries is None or key != self._entries_key:
            rows = [p.entry() for p in self.packs]
            self._entries = torch.tensor(rows, dtype=torch.int64).to(
                self.packs[0].fwd.device)
            self._entries_key = key
            self._max = max(p.numel() for p in self.packs)
        _ops().weight_pack(self._entries, len(self.packs), self._max)
        self._version = self._params_version()

    def _ensure_packed(self):
        if self._version != self._params_version():
            self.pack_weights()

    # ------------------------------------------------------------------ layout
    def to_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        """NCHW-shaped input -> channel-last bf16 with channels padded to 8 (16-byte pixels
        for the first conv's LDS-DMA).  bf16 channels_last input with C % 8 == 0 is used
        zero-copy, and so is a batch from the device input pipeline (``data.engine_input``:
        the generator / gather kernels already wrote this layout)."""
        padded = getattr(x, "_ddlpc_nhwc", None)
        if padded is not None and padded.shape[0] == x.shape[0]:
            return padded
        nd = x.dim()
        perm = (0,) + tuple(range(2, nd)) + (1,)
        xt = x.permute(*perm)
        if xt.is_contiguous() and xt.dtype == torch.bfloat16 and x.shape[1] % 8 == 0:
            return xt
        cl = torch.channels_last if nd == 4 else torch.channels_last_3d
        if not (x.is_contiguous() or x.is_contiguous(memory_format=cl)):
            x = x.contiguous(memory_format=cl)
        return _ops().to_nhwc_bf16(x, 8)

    # ------------------------------------------------------------------ graph
    def features(self, x: torch.Tensor, defer_last: bool = False):
        """Input (NCHW view) -> (last decoder activation, None), channel-last bf16, or with
        ``defer_last`` (pre-BN output, BN statistics) for the fused head kernels.

        A block whose only consumer is one of this engine's transposed convolutions (or the
        head) defers its final BatchNorm + ReLU into that consumer's loads: the activation
        is never materialised, and the consumer's backward kernel also reduces the
        BatchNorm-backward partial sums (SURVEY.md §2.5 K4/K5 fusion)."""
        self._ensure_packed()
        h = self.to_nhwc(x)
        skips = []
        grouped = self.bn_groups >= 1 and self.enc[0].bn1.bn.training
        dskip = self.defer_skip_levels(x) if not grouped else [False] * len(self.enc)
        for lvl, blk in enumerate(self.enc):
            skip, h, s_skip = blk(h, None, True, defer_skip=dskip[lvl])
            skips.append((skip, s_skip))
        n = len(self.dec)
        mode = self.defer_mode if not grouped else "none"    # "all" | "convt" | "none"
        feeds_convt = [pack is not None and mode != "none" for _, pack, _ in self.dec]
        # (grouped: the head's per-group statistics come from its fused TRAINING forward, so a
        # forward under no_grad keeps the last activation materialised)
        defer_last = defer_last and ((self.group_head_defer(x) and torch.is_grad_enabled())
                                     if grouped else mode == "all")
        h, _, s = self.mid(h, None, False, defer=n > 0 and feeds_convt[0])
        for i, ((ub, pack, blk), (skip, s_skip)) in enumerate(zip(self.dec, reversed(skips))):
            if pack is not None:
                up = _ConvTFn.apply(h, ub.up_sample.weight, ub.up_sample.bias, pack, self, s)
            else:
                up = _BilinearFn.apply(h)
            defer = feeds_convt[i + 1] if i + 1 < n else defer_last
            h, _, s = blk(up, skip, False, defer=defer, x2_bn=s_skip)
        return h, s

    def defer_skip_levels(self, x: torch.Tensor) -> List[bool]:
        """Encoder levels whose skip tensor stays pre-BN (BN + ReLU applied on load by the
        decoder's concat conv, forward and weight gradient): 2-D, the skip image at least 16
        wide (the weight-gradient kernels with the X2 prologue) and the concat at most 512
        channels (prologue constants in LDS).  Opt-in: ``engine.defer_skip = True``."""
        if not self.defer_skip or x.dim() != 4:
            return [False] * len(self.enc)
        out = []
        w = x.shape[-1]
        for lvl, blk in enumerate(self.enc):
            ub, _pack, dblk = self.dec[len(self.dec) - 1 - lvl]
            c_up = dblk.conv1.weight.shape[1] - blk.conv2.weight.shape[0]
            c_skip = blk.conv2.weight.shape[0]
            ok = (w >> lvl) >= 16 and c_up % 32 == 0 and c_up + c_skip <= 512 and lvl <= self.defer_skip_max_level
            out.append(bool(ok))
        return out

    def c32_eligible(self, x1: torch.Tensor, x2: Optional[torch.Tensor], cout: int) -> bool:
        """Whether conv3_wgrad takes the 32-output-channel concat kernel for this conv
        (csrc/conv3x3_wgrad_c32.hip conv3_wgrad_c32_plan: 2-D, 64..96 input channels in whole
        32-channel chunks, images >= 16 wide, >= 8 16x16 tiles per CU)."""
        if x2 is None or x1.dim() != 4 or x2.dim() != 4 or cout != 32:
            return False
        n, h, w, c1 = x1.shape
        c2 = x2.shape[-1]
        if c1 % 32 or c2 % 32 or not 64 <= c1 + c2 <= 96 or w < 16:
            return False
        if h * w * max(c1, c2, 32) * 2 >= 2 ** 31:
            return False
        return n * -(-h // 16) * -(-w // 16) >= 8 * int(_ops().set_cu_reserve(-1))

    def group_fused(self, x: torch.Tensor, G: int, cmid: int) -> bool:
        """Whether a DoubleConv on input ``x`` runs the fused BN-group path: 2-D (the
        BN-backward epilogue), a middle width the v3 weight gradient's per-group prologue
        takes (a multiple of 32, images >= 8 wide) and enough pixels per group."""
        if self.group_fuse_min_px is None or x.dim() != 4 or G < 2:
            return False
        n, h, w = x.shape[0], x.shape[1], x.shape[2]
        return (cmid % 32 == 0 and w >= 8 and n % G == 0 and
                (n // G) * h * w >= self.group_fuse_min_px)

    def group_head_defer(self, x: torch.Tensor) -> bool:
        """BN groups: whether the last decoder block's BatchNorm is deferred into the head
        (the C = 32 matrix-core head kernels, group-major; the fused training forward and the
        two-pass backward; pixels per group a multiple of 16)."""
        G = self.bn_groups
        wh = self.head.weight
        if not (self.head_apply and self.head_fused_fwd and G >= 2 and self.group_fuse_min_px is not None):
            return False
        pix = x.shape[0] // G
        for d in x.shape[2:]:
            pix *= d
        return wh.shape[1] == 32 and wh.shape[0] <= 16 and x.shape[0] % G == 0 and pix % 16 == 0

    def bn_groups_supported(self, tile: int) -> bool:
        return bn_groups_supported(self.model, tile)

    def _head_params(self):
        w = self.head.weight
        return w.view(w.shape[0], w.shape[1]), self.head.bias

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        wh, bh = self._head_params()
        if torch.is_grad_enabled() and (wh.requires_grad or x.requires_grad or
                                        any(p.requires_grad for p in self.model.parameters())):
            # differentiable logits (rare: training uses loss_and_correct)
            a, _ = self.features(x)
            logits = torch.einsum("n...c,kc->n...k", a.float(), wh) + bh
            return _nhwc_shape_to_nchw(logits)
        a, s = self.features(x, defer_last=True)
        return _ops().head_logits(a, wh.detach().contiguous(), bh.detach(), s)

    def loss_and_correct(self, x: torch.Tensor, y: torch.Tensor, ignore_index: int = -100):
        """-> (mean cross-entropy over the batch's pixels, correct-pixel count).  With
        ``bn_groups`` = G >= 1 (training) the batch is G equal micro-batches with their own
        BatchNorm statistics; the running statistics are updated once per micro-batch, in
        order, after the forward (bit-for-bit the update sequence of G forwards)."""
        G = self.bn_groups if self.enc[0].bn1.bn.training else 0
        if G >= 1:
            if x.shape[0] % G:
                raise ValueError(f"bn_groups={G} must divide the batch ({x.shape[0]})")
            self.bn_defer_prepare(1, G)
        a, s = self.features(x, defer_last=True)
        wh, bh = self._head_params()
        out = _HeadCEFn.apply(a, wh, bh, y.contiguous(), ignore_index, self, s)
        if G >= 1:
            self.bn_defer_apply(G)
        return out
