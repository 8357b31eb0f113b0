"""Bucketed data-parallel gradient reducer, overlapped with backward.

Replaces the reference's star exchange: workers encode
their accumulated gradients, send them to rank 0 over TCP, rank 0 merges, re-encodes and
sends back, everyone steps Adam (ref.py:255-556).  That serialises a 2*M*msg transfer
through one link and round-trips every tensor through the host.

MI355X design:

* gradients are views into ONE flat fp32 buffer (``FlatParams``); buckets are contiguous
  slices of it in backward order, sized by ``bucket_mb`` (few, large: on 7 point-to-point
  xGMI links per GPU a ring all-reduce is per-link bound, and per-collective latency is
  tens of µs, so 3-5 buckets of ~8 MB beat many small ones);
* ``register_post_accumulate_grad_hook`` marks parameters ready; when the LAST
  micro-batch's backward completes a bucket, its collective is launched immediately
  (async) so it runs on RCCL's own stream while backward continues on the compute
  stream: the deep decoder/bottleneck gradients (most of the bytes) reduce while the
  high-resolution encoder layers are still in backward;
* accumulation micro-batches (``frequency_sending_gradients``, ref.py:685/759) launch
  nothing (no_sync semantics);
* ``finish()`` makes the compute stream wait for every bucket (no host sync) before the
  optimizer step;
* reduction: correct mean (pre-scaled by 1/W, then SUM), ``sum``, or ``reference`` (the
  reference's skewed weights; for W=2 that is a plain sum);
* optional lossy codec (fp16/int8 absmax, ref.py:25) as an all-gather of packed payloads
  + scales, decoded and summed in rank order (``parallel.codec``; fused HIP kernels on GPU);
* optional bf16 wire format (``wire_dtype="bf16"``): half the bytes of the fp32
  all-reduce — an all-to-all of bf16 chunks (the reduce-scatter's transport) launched
  asynchronously from backward, then in ``finish()`` a rank-ordered fp32 sum of the owned
  chunk and an all-gather of the sums.  LOSSY: each rank's gradient is rounded to bf16
  before the exchange and the reduced gradient is rounded to bf16 again before it is
  copied back into the fp32 grad buffer (every rank receives identical bits).  For slow
  links (the reference's "PCs over Ethernet" setting) this halves the bytes on the wire.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import codec as C
from .flat import FlatParams


class _Bucket:
    __slots__ = ("idx", "start", "end", "params", "pending", "work", "payload", "scales",
                 "gathered", "launched", "wire", "ev")

    def __init__(self, idx, start, end, params):
        self.idx, self.start, self.end, self.params = idx, start, end, params
        self.pending = len(params)
        self.work = None
        self.payload = self.scales = self.gathered = None
        self.launched = False
        self.wire = None                 # bf16 wire buffers (send, recv, owned chunk, out)
        self.ev = None                   # comm proxy: (ready, start, end) events


class GradBucketReducer:
    def __init__(self, flat: FlatParams, group=None, bucket_mb: float = 8.0,
                 reduce: str = "mean", grad_codec: str = "none", codec_scale: str = "bucket",
                 overlap: bool = True, use_hooks: bool = True, wire_dtype: str = "fp32",
                 proxy: int = 0, cuts: Optional[List[int]] = None):
        if wire_dtype not in ("fp32", "bf16"):
            raise ValueError(f"wire_dtype={wire_dtype!r}")
        self.flat = flat
        self.wire_dtype = wire_dtype
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.backend = dist.get_backend(group) if dist.is_initialized() else None
        # comm proxy (single GPU; ``proxy`` = the world size it stands in for): every
        # bucket's collective is replaced by ``comm_proxy`` — 16 streaming workgroups (an
        # RCCL-like channel count) sweeping the bucket twice (reduce-scatter + all-gather
        # passes, values unchanged) — on a dedicated comm stream, launched at the same
        # readiness points as the real collective.  It measures how fast a collective
        # launched mid-backward gets CUs next to the persistent kernels.
        self.proxy = int(proxy) if self.world == 1 else 0
        self.proxy_stream = None
        self.proxy_log: List[Tuple[int, float, float]] = []
        if self.proxy:
            if grad_codec != "none" or wire_dtype != "fp32":
                raise ValueError("comm proxy: plain fp32 all-reduce only")
            self.world = 2                       # every rank path below behaves as DP ...
            reduce = "sum"                       # ... with the identity as the reduction
            self.proxy_stream = torch.cuda.Stream(flat.grad_buf.device)
        self.reduce, self.codec, self.codec_scale = reduce, grad_codec, codec_scale
        self.overlap = overlap and not (grad_codec != "none" and codec_scale == "global")
        if reduce == "mean":
            self.weight = 1.0 / self.world
        elif reduce == "sum":
            self.weight = 1.0
        elif reduce == "reference":
            self.weight = C.reference_weights(self.world)[self.rank]
        else:
            raise ValueError(reduce)
        # cuts: bucket boundaries as indices into flat.order (``parallel.bucket_plan``, the
        # readiness-aware plan); None = cut by size only
        self.cuts = list(cuts) if cuts is not None else None
        self.buckets = self._make_buckets(bucket_mb)
        self._bucket_of: Dict[int, _Bucket] = {}
        for b in self.buckets:
            for p in b.params:
                self._bucket_of[id(p)] = b
        # readiness is armed explicitly per accumulation window: only ``prepare(sync=True)``
        # (the window's last micro-batch) arms it and ``finish()`` disarms it, so a fresh
        # reducer — or one between windows — never launches a collective on a partially
        # accumulated gradient (ref.py:756-766: no exchange until the 50th micro-batch)
        self._sync = False
        self._seen = set()
        self._hooks = []
        # readiness: autograd post-accumulate hooks (stock PyTorch modules), or — with
        # use_hooks=False — ONLY explicit mark_ready() calls from kernels that write .grad
        # directly (the HIP engine).  Never both: autograd still runs the AccumulateGrad
        # nodes of such parameters (with no gradient), which would count them twice and
        # launch a bucket before its last gradient is written.
        if self.world > 1 and use_hooks and not self.proxy:
            for p in flat.order:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad_ready))
        self.stats = {"buckets": len(self.buckets), "launched_in_backward": 0}
        # readiness calibration (``start_calibration``): per-parameter gradient-complete times
        # of one synchronised step, relative to its backward start (Trainer.calibrate_bucket_plan)
        self._index = {id(p): i for i, p in enumerate(flat.order)}
        self._calib: Optional[Dict] = None
        self._bwd_start = None

    # ------------------------------------------------------------------ timing marks
    def _now(self):
        """A timing mark on the current stream (hipEvent), or the host clock on CPU (gloo: hooks
        fire synchronously on the host)."""
        dev = self.flat.grad_buf.device
        if dev.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(dev))
            return e
        import time
        return time.perf_counter()

    @staticmethod
    def _ms(a, b) -> float:
        return a.elapsed_time(b) if isinstance(a, torch.cuda.Event) else (b - a) * 1e3

    def mark_backward_start(self):
        """Called right before the synchronised micro-batch's backward is queued (its forward
        kernels are ahead of it on the stream): the zero of the readiness times."""
        if self._sync and (self._calib is not None or self.proxy):
            self._bwd_start = self._now()

    def start_calibration(self):
        self._calib = {"ready": {}, "end": None}

    def stop_calibration(self) -> Tuple[List[float], float]:
        """-> (ready ms of every parameter in flat order, backward ms) of the calibrated step,
        both measured from the backward start (synchronises).  A parameter never reported ready
        counts as ready at the backward's end."""
        cal, self._calib = self._calib, None
        if cal is None or self._bwd_start is None or cal["end"] is None:
            raise RuntimeError("calibration: no synchronised step was recorded")
        t0 = self._bwd_start
        if isinstance(t0, torch.cuda.Event):
            cal["end"].synchronize()
        bwd = self._ms(t0, cal["end"])
        ready = [bwd] * len(self.flat.order)
        for i, ev in cal["ready"].items():
            ready[i] = min(bwd, max(0.0, self._ms(t0, ev)))
        return ready, bwd

    # ------------------------------------------------------------------ setup
    def _make_buckets(self, bucket_mb: float) -> List[_Bucket]:
        order = self.flat.order
        if self.cuts is not None:
            c = self.cuts
            if c[0] != 0 or c[-1] != len(order) or any(b <= a for a, b in zip(c[:-1], c[1:])):
                raise ValueError(f"bucket cuts {c} do not partition {len(order)} parameters")
            out = []
            for a, b in zip(c[:-1], c[1:]):
                ps = order[a:b]
                out.append(_Bucket(len(out), self.flat.span(ps[0])[0], self.flat.span(ps[-1])[1], ps))
            return out
        cap = max(1, int(bucket_mb * (1 << 20) // 4))
        buckets, cur, start = [], [], None
        end = 0
        for p in self.flat.order:
            a, b = self.flat.span(p)
            if start is None:
                start = a
            if cur and (b - start) > cap:
                buckets.append(_Bucket(len(buckets), start, end, cur))
                cur, start = [], a
            cur.append(p)
            end = b
        if cur:
            buckets.append(_Bucket(len(buckets), start, end, cur))
        # last bucket extends over trailing alignment padding (harmless zeros)
        return buckets

    def bucket_ranges(self) -> List[Tuple[int, int]]:
        return [(b.start, b.end) for b in self.buckets]

    # ------------------------------------------------------------------ per step
    @contextlib.contextmanager
    def no_sync(self):
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev

    def prepare(self, sync: bool = True):
        """Call before each micro-batch backward: ``sync`` only on the last one of the
        accumulation window (arms the bucket launches; ``finish()`` disarms them)."""
        self._sync = sync
        if sync:
            self._seen = set()
            for b in self.buckets:
                b.pending = len(b.params)
                b.work = None
                b.launched = False
                b.payload = b.scales = b.gathered = None

    def mark_ready(self, p):
        """Readiness notification from kernels that write .grad directly (HIP engine)."""
        self._on_grad_ready(p)

    def _on_grad_ready(self, p):
        if not self._sync or not self.overlap:
            return
        b = self._bucket_of.get(id(p))
        if b is None or id(p) in self._seen:       # a parameter counts once per step
            return
        self._seen.add(id(p))
        if self._calib is not None:
            self._calib["ready"][self._index[id(p)]] = self._now()
        b.pending -= 1
        if b.pending == 0 and not b.launched:
            self._launch(b)
            self.stats["launched_in_backward"] += 1

    def _seg(self, b: _Bucket) -> torch.Tensor:
        return self.flat.grad_buf[b.start:b.end]

    def _launch(self, b: _Bucket):
        b.launched = True
        g = self._seg(b)
        if self.proxy:
            self._launch_proxy(b, g)
            return
        if self.codec == "none":
            # pre-scaled SUM on every backend (exact for power-of-two world sizes; no
            # dependence on the collective library's AVG support)
            if self.weight != 1.0:
                g.mul_(self.weight)
            if self.wire_dtype == "bf16":
                self._launch_bf16(b, g)
                return
            b.work = dist.all_reduce(g, group=self.group, async_op=True)
            return
        # lossy codec: encode -> all_gather(payload, scales) -> decode+sum at finish()
        segs = self._codec_segments(b)
        from ..ops import codec_ops
        b.payload, b.scales = codec_ops.encode_segments(g, segs, self.codec)
        b.gathered = ([torch.empty_like(b.payload) for _ in range(self.world)],
                      [torch.empty_like(b.scales) for _ in range(self.world)])
        w1 = dist.all_gather(b.gathered[0], b.payload, group=self.group, async_op=True)
        w2 = dist.all_gather(b.gathered[1], b.scales, group=self.group, async_op=True)
        b.work = (w1, w2)

    PROXY_BLOCKS = 16                    # RCCL-like channel count

    def _launch_proxy(self, b: _Bucket, g: torch.Tensor):
        cur = torch.cuda.current_stream(g.device)
        if b.ev is None:
            b.ev = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
        ready, start, end = b.ev
        ready.record(cur)                    # gradients complete on the producing stream
        st = self.proxy_stream
        st.wait_stream(cur)                  # as RCCL's stream waits on the caller's
        with torch.cuda.stream(st):
            start.record(st)
            from ..ops import _ext
            # two sweeps: the reduce-scatter's and the all-gather's pass over the bucket
            _ext.ops().comm_proxy(g, self.PROXY_BLOCKS, 2)
            end.record(st)
        b.work = ("proxy", end)

    def proxy_times(self) -> List[Dict[str, float]]:
        """Per bucket of the last synchronised step: ms from gradients-ready to the proxy
        collective's start and end (synchronises on the events)."""
        out = []
        for b in self.buckets:
            if b.ev is None:
                continue
            ready, start, end = b.ev
            end.synchronize()
            rec = {"bucket": b.idx, "mb": round((b.end - b.start) * 4 / 2**20, 2),
                   "ready_to_start_ms": ready.elapsed_time(start),
                   "ready_to_end_ms": ready.elapsed_time(end),
                   "kernel_ms": start.elapsed_time(end)}
            if isinstance(self._bwd_start, torch.cuda.Event):
                # bucket collective end measured from the backward start (the plan's zero)
                rec["end_from_backward_start_ms"] = self._bwd_start.elapsed_time(end)
            bwd = getattr(self, "_bwd_end", None)
            if bwd is not None:
                bwd.synchronize()
                # > 0: the bucket's collective ended after backward (exposed)
                rec["end_after_backward_ms"] = bwd.elapsed_time(end)
            out.append(rec)
        return out

    def _launch_bf16(self, b: _Bucket, g: torch.Tensor):
        """bf16 transport, first half: the all-to-all of bf16 chunks, left in flight (its
        wait, the fp32 rank-order sum and the all-gather run in ``finish()``, so backward is
        never blocked by the exchange — on gloo a wait here would stall the host)."""
        n, W = g.numel(), self.world
        chunk = -(-n // W)
        if b.wire is None:
            send = torch.zeros(chunk * W, dtype=torch.bfloat16, device=g.device)
            b.wire = (send, torch.empty_like(send),
                      torch.empty(chunk, dtype=torch.bfloat16, device=g.device),
                      torch.empty_like(send))
        send, recv, own, out = b.wire
        send[:n].copy_(g)
        b.work = ("a2a", dist.all_to_all_single(recv, send, group=self.group, async_op=True))

    def _finish_bf16(self, b: _Bucket):
        """bf16 transport, second half: wait the all-to-all, sum the owned chunk in fp32 in
        rank order, launch the all-gather of the sums (waited by the caller)."""
        _, recv, own, out = b.wire
        chunk = own.numel()
        b.work[1].wait()
        own.copy_(recv.view(self.world, chunk).float().sum(0))
        b.work = ("bf16", dist.all_gather_into_tensor(out, own, group=self.group,
                                                      async_op=True))

    def _codec_segments(self, b: _Bucket) -> List[Tuple[int, int]]:
        if self.codec_scale == "tensor":
            return [(s - b.start, e - b.start) for s, e in (self.flat.span(p) for p in b.params)]
        return [(0, b.end - b.start)]

    def finish(self):
        """Complete all reductions (launch stragglers); compute stream waits, host does not."""
        if self.world == 1:
            return
        if self._calib is not None and self._calib["end"] is None:
            self._calib["end"] = self._now()          # backward's end (before the stragglers)
        if self.proxy:
            # backward's end on the compute stream (proxy_times: bucket end vs backward end)
            if getattr(self, "_bwd_end", None) is None:
                self._bwd_end = torch.cuda.Event(enable_timing=True)
            self._bwd_end.record(torch.cuda.current_stream(self.flat.grad_buf.device))
        if self.codec != "none" and self.codec_scale == "global":
            self._finish_global_codec()
            self._sync = False
            return
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        for b in self.buckets:                      # bf16 wire: all-gathers in bucket order
            if isinstance(b.work, tuple) and b.work[0] == "a2a":
                self._finish_bf16(b)
        for b in self.buckets:
            if b.work is None:
                continue
            if isinstance(b.work, tuple) and b.work[0] == "proxy":
                torch.cuda.current_stream(self.flat.grad_buf.device).wait_event(b.work[1])
            elif isinstance(b.work, tuple) and b.work[0] == "bf16":
                b.work[1].wait()
                g = self._seg(b)
                g.copy_(b.wire[3][:g.numel()])
            elif isinstance(b.work, tuple):
                for w in b.work:
                    w.wait()
                self._decode_bucket(b)
            else:
                b.work.wait()
            b.work = None
        self._sync = False                          # disarmed until the next window's last micro-batch

    def _decode_bucket(self, b: _Bucket):
        from ..ops import codec_ops
        g = self._seg(b)
        segs = self._codec_segments(b)
        weights = (C.reference_weights(self.world) if self.reduce == "reference"
                   else [self.weight] * self.world)
        codec_ops.decode_sum_segments(g, b.gathered[0], b.gathered[1], segs, self.codec,
                                      weights)
        b.gathered = b.payload = b.scales = None

    def _finish_global_codec(self):
        """Reference-parity mode: one absmax over the WHOLE gradient (ref.py:328-340)."""
        from ..ops import codec_ops
        g = self.flat.grad_buf
        segs = [(0, g.numel())]
        payload, scales = codec_ops.encode_segments(g, segs, self.codec)
        qs = [torch.empty_like(payload) for _ in range(self.world)]
        ss = [torch.empty_like(scales) for _ in range(self.world)]
        dist.all_gather(qs, payload, group=self.group)
        dist.all_gather(ss, scales, group=self.group)
        weights = (C.reference_weights(self.world) if self.reduce == "reference"
                   else [self.weight] * self.world)
        codec_ops.decode_sum_segments(g, qs, ss, segs, self.codec, weights)

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
