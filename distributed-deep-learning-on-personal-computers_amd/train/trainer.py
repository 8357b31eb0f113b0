"""``train()`` / ``validate()`` entrypoints and the data-parallel training step.

Reference training drivers: rank 0 ("server", ref.py:690-790)
and rank>0 ("worker", ref.py:792-895) run the same loop — forward, ``CrossEntropyLoss``,
``backward()`` accumulating into ``.grad`` WITHOUT zero_grad, and every
``frequency_sending_gradients``-th micro-batch a gradient exchange + ``optimizer.step()``
+ ``zero_grad()`` (ref.py:750-766, 864-879).

This trainer keeps those semantics — ``accum_steps`` micro-batches of ``batch_per_gpu``
per optimizer step, gradients accumulated in place, one synchronous exchange per step so
every rank applies identical gradients — with the MI355X machinery underneath:

* one process per GPU, ``torch.distributed`` over RCCL (gloo on CPU);
* the U-Net hot path in hand-written HIP kernels (``impl="hip"``: NHWC bf16 MFMA
  convolutions with fused BN/ReLU/pool/concat, fused head+CE) or stock PyTorch
  (``impl="torch"``: the CPU path and the MIOpen in-house baseline);
* flat fp32 parameters/gradients, a bucketed all-reduce launched from backward hooks on
  the last micro-batch only, one fused Adam launch;
* metrics accumulate on the device and are reduced across ranks only at log points.
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..config import TrainConfig
from ..data import ShardedSampler, SyntheticTiles, TileDataset
from ..models.unet import UNet
from ..ops import _ext
from ..ops.adam import FlatAdam
from ..parallel import (GradBucketReducer, assert_replicas_identical, broadcast_buffers,
                        broadcast_module, broadcast_tensors, flatten_module, init_distributed)
from ..utils.metrics import DeviceMeter, RunLogger, dump_pngs
from ..utils.tracing import PhaseTimer, StepProfiler, enable_ranges, trace_range
from .checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint


def resolve_impl(impl: str, device: torch.device, dtype: str = "bf16") -> str:
    """``auto``: the operator engine for bf16 compute, stock ``nn`` modules for fp32 compute
    (the reference's precision, ref.py:702-704).  The choice is the compute precision, not
    the device: the engine's ``torch.ops.ddlpc`` operators dispatch by tensor device
    (gfx950 kernels for GPU tensors, the C++ reference kernels of ``csrc/cpu_ref.cpp`` for
    CPU tensors).  ``hip`` with fp32 is rejected by the config."""
    del device
    if impl == "auto":
        return "hip" if dtype == "bf16" else "torch"
    if impl == "hip" and dtype != "bf16":
        raise ValueError("impl='hip' computes in bf16 (dtype='fp32' needs impl='torch')")
    return impl


class Trainer:
    def __init__(self, cfg: TrainConfig, device: Optional[str] = None):
        cfg.validate()
        self.cfg = cfg
        self.info = init_distributed(cfg.backend, cfg.timeout_s, device)
        self.device = self.info.device
        self.rank, self.world = self.info.rank, self.info.world_size
        torch.manual_seed(cfg.seed)                  # identical init on every rank ...
        model = UNet.from_config(cfg.model).to(self.device)
        self.impl = resolve_impl(cfg.impl, self.device, cfg.dtype)
        self.model = model
        if self.device.type == "cuda" and self.impl == "torch":
            # MIOpen NHWC / NDHWC path (baseline)
            model.to(memory_format=torch.channels_last if cfg.model.dims == 2
                     else torch.channels_last_3d)
        self.flat = flatten_module(model)
        broadcast_module(model, src=0)               # ... and rank 0 is authoritative
        if self.impl == "hip":
            _ext.ops()                               # fail loudly if kernels are missing
            model.to_hip()
            model._engine.recompute = int(cfg.recompute)
        self.optimizer = FlatAdam(self.flat, lr=cfg.lr, betas=cfg.betas, eps=cfg.eps,
                                  weight_decay=cfg.weight_decay,
                                  use_hip=(self.impl == "hip"))
        if self.impl == "hip":
            self.optimizer.weight_pack = model._engine.pack_weights
        # optional CU reservation for collectives (persistent grids sized to num_cus - k).
        # Default 0: the comm proxy measured a bucket collective launched mid-backward
        # starting within ~20 us without any reservation (the side stream's weight-gradient
        # workgroups keep releasing slots), while 8 reserved CUs cost 5% of the step
        # (persistent grids lose their even split of tiles over 256 CUs)
        if cfg.comm_proxy and (self.impl != "hip" or self.world > 1):
            raise ValueError("comm_proxy: single-GPU HIP runs only (it stands in for RCCL)")
        dp = self.world > 1 or cfg.comm_proxy > 0
        self.reserve_cus = max(0, cfg.reserve_cus)
        if self.impl == "hip":
            self.grid_cus = int(_ext.ops().set_cu_reserve(self.reserve_cus))
        self.reducer = None
        if dp:
            self.reducer = self._make_reducer(cfg.bucket_mb)
        if self.impl == "hip":
            # kernels write gradients straight into the flat grad buffer and trigger the
            # reducer's buckets themselves (no autograd accumulate pass)
            model._engine.enable_direct_grads(
                self.reducer.mark_ready if self.reducer is not None else None)
        self.autocast = (self.device.type == "cuda" and self.impl == "torch"
                         and cfg.dtype == "bf16")
        self.meter = DeviceMeter(self.device)
        self.logger = RunLogger(cfg.log_dir, self.rank, cfg.grad_codec)
        if cfg.trace_ranges:
            enable_ranges(True)
        self.phases = PhaseTimer(self.device) if cfg.phase_timers else None
        self.profiler = StepProfiler(cfg.profile_dir, self.rank, active=cfg.profile_steps)
        # host run-ahead bound: before queueing a step the host waits until the step
        # ``max_inflight`` steps back has finished on the GPU.  Unbounded run-ahead queues
        # thousands of cross-stream barrier packets (weight-gradient side stream); measured:
        # some processes then ran 2-4x slower (1,472-2,703 vs 5,975 images/s, same box)
        # while a bounded queue keeps the GPU fed (>= one whole step queued).
        self.max_inflight = int(os.environ.get("DDLPC_MAX_INFLIGHT", "2"))
        self._inflight: List[torch.cuda.Event] = []
        self.step_count = 0
        self.micro_count = 0
        self.micro_streams = self._resolve_micro_streams()
        self._mstreams: List[torch.cuda.Stream] = []     # concurrent micro-batch streams
        self.ms_graph = True                               # ... each replaying its own graph
        self._ms_meters: List[DeviceMeter] = []
        self._ms_graphs, self._ms_warm, self._ms_static = [], [], []
        self.ms_host_s = 0.0
        self._mbufs: List[torch.Tensor] = []               # their extra gradient buffers
        self._mviews: List[list] = []
        self._flat_views = None
        self._graphs: Dict[str, "torch.cuda.CUDAGraph"] = {}   # hipGraphs (cfg.hip_graph)
        self._graph_warm: Dict[str, int] = {}
        self._static = None
        self.epoch = 0
        self.epoch_step = 0              # optimizer steps done in the current epoch
        self.train_set, self.test_set = self._build_data()
        self.sampler = ShardedSampler(len(self.train_set), self.rank, self.world,
                                      shard=cfg.shard_data, shuffle=cfg.shuffle, seed=cfg.seed)
        if cfg.resume:
            path = latest_checkpoint(cfg.ckpt_dir) if cfg.resume == "auto" else cfg.resume
            exists = bool(path) and os.path.exists(path)
            if cfg.resume != "auto":
                # an explicit path must exist on rank 0 (its state is broadcast below); other
                # ranks may lack the file (no shared filesystem) and receive rank 0's state.
                # Every rank learns rank 0's verdict, so a bad path fails the whole job at
                # once instead of leaving ranks > 0 blocked in the state broadcast
                found = torch.tensor([1.0 if exists else 0.0], device=self.device)
                if self.world > 1:
                    dist.broadcast(found, src=0)
                if found.item() == 0.0:
                    raise FileNotFoundError(f"resume checkpoint not found on rank 0: {cfg.resume}")
            if exists:
                self.load(path)
            # only rank 0 writes checkpoints: on machines without a shared filesystem the
            # other ranks find none, so rank 0's restored state is authoritative
            self._broadcast_state()

    def _make_reducer(self, bucket_mb: float, cuts: Optional[List[int]] = None) -> GradBucketReducer:
        """The gradient reducer; ``cuts`` given = those bucket cuts (a calibrated plan),
        else the configured plan (readiness model / size)."""
        c = self.cfg
        if cuts is None:
            self.bucket_plan = None
        if cuts is None and c.bucket_plan == "readiness":
            from ..parallel.bucket_plan import plan_for_model
            world = self.world if self.world > 1 else max(2, c.comm_proxy)
            self.bucket_plan = plan_for_model(
                self.model, self.flat.order, c.model, c.tile, c.batch_per_gpu, world,
                self.info.backend if self.world > 1 else "nccl", bucket_mb,
                wire_bytes=2 if c.wire_dtype == "bf16" else 4)
            cuts = self.bucket_plan.cuts
        return GradBucketReducer(self.flat, bucket_mb=bucket_mb, reduce=c.reduce,
                                 grad_codec=c.grad_codec, codec_scale=c.codec_scale,
                                 overlap=c.overlap_comm, use_hooks=(self.impl != "hip"),
                                 wire_dtype=c.wire_dtype,
                                 proxy=c.comm_proxy if self.world == 1 else 0, cuts=cuts)

    def calibrate_bucket_plan(self, micro_batches) -> Optional[Dict]:
        """Re-plan the readiness-aware buckets from ONE measured step (untimed; call after
        warm-up): every parameter's gradient-complete time and the backward time replace the
        FLOP-rate model of ``plan_for_model``.  Every rank cuts identically (MAX of the per-rank
        timings).  Under the single-GPU comm proxy the collective cost model (latency,
        bandwidth) is fitted to the proxy collectives of the same step.  Returns a summary."""
        c = self.cfg
        r = self.reducer
        if r is None or c.bucket_plan != "readiness" or getattr(self, "bucket_plan", None) is None:
            return None
        from ..parallel import bucket_plan as BP
        r.start_calibration()
        self.train_step(micro_batches)
        ready_ms, bwd_ms = r.stop_calibration()
        if self.world > 1:
            dev = self.device if dist.get_backend() == "nccl" else torch.device("cpu")
            t = torch.tensor(ready_ms + [bwd_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            vals = t.tolist()
            ready_ms, bwd_ms = vals[:-1], vals[-1]
        world = self.world if self.world > 1 else max(2, c.comm_proxy)
        gpu = (self.info.backend if self.world > 1 else "nccl") == "nccl"
        gbps = BP.XGMI_RING_GBPS if gpu else BP.GLOO_GBPS
        lat_us = BP.XGMI_LAT_US if gpu else BP.GLOO_LAT_US
        fitted = None
        if r.proxy:
            recs = r.proxy_times()
            fit = BP.fit_collective_model([x["mb"] * 2**20 for x in recs],
                                          [x["kernel_ms"] for x in recs], world)
            if fit is not None:
                gbps, lat_us = fit
                fitted = {"gbps": round(gbps, 2), "lat_us": round(lat_us, 1)}
        wire = 2 if c.wire_dtype == "bf16" else 4
        nbytes = [float(p.numel() * wire) for p in self.flat.order]
        plan = BP.plan_buckets(nbytes, [v / max(bwd_ms, 1e-9) for v in ready_ms], bwd_ms,
                               world, gbps, lat_us, c.bucket_mb * (1 << 20) * wire / 4.0)
        plan.calibrated = True
        self.bucket_plan = plan
        r.remove_hooks()
        self.reducer = self._make_reducer(c.bucket_mb, cuts=plan.cuts)
        if self.impl == "hip":
            self.model._engine.enable_direct_grads(self.reducer.mark_ready)
        return {"backward_ms": round(bwd_ms, 3), "buckets": len(plan.cuts) - 1,
                "bucket_mb": [round(sum(nbytes[a:b]) / 2**20, 2)
                              for a, b in zip(plan.cuts[:-1], plan.cuts[1:])],
                "predicted_end_ms": [round(v, 3) for v in plan.bucket_done_ms],
                "predicted_exposed_ms": round(plan.exposed_ms, 3), "collective_fit": fitted}

    def set_bucket_mb(self, bucket_mb: float) -> int:
        """Re-bucket the gradient reducer between steps (bucket-size sweeps);
        returns the number of buckets."""
        if self.reducer is None:
            return 0
        self.reducer.remove_hooks()
        self.cfg.bucket_mb = bucket_mb
        self.reducer = self._make_reducer(bucket_mb)
        if self.impl == "hip":
            self.model._engine.enable_direct_grads(self.reducer.mark_ready)
        return len(self.reducer.buckets)

    def _broadcast_state(self):
        """Rank 0's parameters, buffers, Adam moments and step counters -> every rank."""
        if self.world == 1:
            return
        broadcast_module(self.model, src=0)
        broadcast_tensors([self.optimizer.exp_avg, self.optimizer.exp_avg_sq], src=0)
        cnt = torch.tensor([self.epoch, self.step_count, self.micro_count, self.epoch_step,
                            self.optimizer.step_count], dtype=torch.int64, device=self.device)
        dist.broadcast(cnt, src=0)
        (self.epoch, self.step_count, self.micro_count, self.epoch_step,
         opt_steps) = (int(v) for v in cnt.tolist())
        self.optimizer.step_count = opt_steps
        if self.optimizer._dev_scal is not None:
            self.optimizer._dev_scal[0] = float(opt_steps)
        if self.model._engine is not None:
            self.model._engine.pack_weights()

    # ------------------------------------------------------------------ data
    def _build_data(self):
        """Datasets that produce device batches directly on a GPU: the
        synthetic generator renders in HBM, a real dataset is uploaded once as uint8."""
        c = self.cfg
        cuda = self.device.type == "cuda"
        layout = "engine" if self.impl == "hip" else "nchw"
        if c.data == "vaihingen_dir":
            if not c.data_dir:
                raise ValueError("data=vaihingen_dir needs data_dir")
            tr, te = TileDataset.from_dir(c.data_dir, c.test_holdout)
            if cuda and c.data_on_device:
                budget = None if c.data_hbm_gb is None else int(c.data_hbm_gb * 2**30)
                tr = tr.to_device(self.device, layout, budget)
                te = te.to_device(self.device, layout, budget) if te is not None else None
            return tr, te
        n_total = c.num_samples + c.test_holdout
        dev = self.device if (cuda and c.data_on_device) else None
        full = SyntheticTiles(n_total, c.tile, c.model.out_classes, c.model.in_channels,
                              seed=c.seed, dims=c.model.dims, device=dev, layout=layout)
        return _Subset(full, 0, c.num_samples), _Subset(full, c.num_samples, n_total)

    def _to_device(self, x, y):
        if x.device == self.device and getattr(x, "_ddlpc_nhwc", None) is not None:
            return x, y.to(self.device, non_blocking=True)     # engine layout, already in HBM
        x = x.to(self.device, non_blocking=True)
        y = y.to(self.device, non_blocking=True)
        if self.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last if x.dim() == 4
                             else torch.channels_last_3d)
            if self.impl == "hip":
                x = x.to(torch.bfloat16)
        return x, y

    # ------------------------------------------------------------------ step
    def _micro(self, x, y, sync: bool):
        if self.reducer is not None:
            self.reducer.prepare(sync=sync)
        ctx = (torch.autocast("cuda", dtype=torch.bfloat16) if self.autocast
               else contextlib.nullcontext())
        with ctx:
            loss, correct = self.model.loss_and_correct(x, y)
        if sync and self.reducer is not None:
            self.reducer.mark_backward_start()
        loss.backward()
        self.meter.add(loss, correct, y.numel())
        self.micro_count += 1
        return loss

    # ------------------------------------------------------------------ concurrent micro-batches
    def _concurrent_ok(self, n_micro: int) -> bool:
        return (self.micro_streams > 1 and n_micro > 1 and self.impl == "hip"
                and self.device.type == "cuda")

    SMALL_MICRO_PIXELS = 4 * 256 * 256          # one 512² image, four 256² ones

    def _resolve_micro_streams(self) -> int:
        """cfg.micro_streams (-1 = auto): 3 concurrent micro-batch streams when micro-batches
        are small (<= SMALL_MICRO_PIXELS) and accumulated, else 1.  Measured at 512² batch 1,
        50 micro-batches, with per-stream graphs: 1 / 2 / 3 / 4 / 6 streams = 356 / 520 /
        638 / 513 / 646 images/s — 3 streams plus the caller's fill the process's 4 hardware
        queues (GPU_MAX_HW_QUEUES); a 4th stream shares one and serialises."""
        c = self.cfg
        if c.micro_streams >= 0:
            return max(1, c.micro_streams)
        px = c.batch_per_gpu * c.tile ** c.model.dims
        small = px <= self.SMALL_MICRO_PIXELS
        return 3 if (c.accum_steps > 1 and small and self.impl == "hip"
                     and self.device.type == "cuda") else 1

    def _grad_views(self, buf: torch.Tensor):
        from ..parallel.flat import FlatParams
        f = self.flat
        return [FlatParams._view(buf, f.offsets[id(p)], p) for p in f.order]

    def _ms_streams(self, K: int, cur) -> List[torch.cuda.Stream]:
        """K plain HIP micro-batch streams.  (CU-masked streams, one chip slice each, were
        measured 2-3x slower than plain ones: 171 vs 515 images/s at K = 4, docs/PERF.md.)"""
        if len(self._mstreams) != K:
            self._mstreams = [torch.cuda.Stream(self.device) for _ in range(K)]
            self._ms_graphs, self._ms_warm, self._ms_static = [None] * K, [0] * K, [None] * K
        return self._mstreams

    def _ms_buffers(self, K: int):
        while len(self._mbufs) < K - 1:
            self._mbufs.append(torch.zeros_like(self.flat.grad_buf))
            self._mviews.append(self._grad_views(self._mbufs[-1]))
        if self._flat_views is None:
            self._flat_views = self._grad_views(self.flat.grad_buf)
        while len(self._ms_meters) < K:
            self._ms_meters.append(DeviceMeter(self.device))
        return [self._flat_views] + self._mviews[:K - 1]

    def _ms_enter(self, K: int):
        """Per-window setup: the weight-gradient side stream off (returns its state)."""
        eng = self.model._engine
        state = eng.side is not None
        eng.set_side_stream(False)
        return state

    def _ms_exit(self, state):
        eng = self.model._engine
        eng.bn_defer_j = None
        for p, g in zip(self.flat.order, self._flat_views):
            p.grad = g
        eng.set_side_stream(state)

    def _ms_finish(self, K: int, n: int):
        """After the streams joined: extra gradient buffers into the flat one (stream
        order), per-stream meters into the trainer's."""
        for b in self._mbufs[:K - 1]:
            self.flat.grad_buf.add_(b)
            b.zero_()
        for m in self._ms_meters[:K]:
            self.meter.buf += m.buf
            m.buf.zero_()
        self.micro_count += n

    def _ms_body(self, k: int, x, y):
        loss, correct = self.model.loss_and_correct(x, y)
        loss.backward()
        self._ms_meters[k].add(loss, correct, y.numel())

    def _concurrent_micros(self, mbs: List[Tuple[torch.Tensor, torch.Tensor]]):
        """Accumulation micro-batches on ``micro_streams`` HIP streams at once.

        The reference's regime (batch 1 per GPU, 50 accumulated micro-batches per exchange,
        ref.py:685-687,750-766) leaves the GPU mostly idle inside each micro-batch: the deep
        layers of one 512² image are a few hundred pixels.  Independent micro-batches fill
        it: micro-batch j runs forward AND backward on stream j % K (autograd keeps a
        backward on its forward's stream; a stream's micro-batches follow each other), with
          * its own gradient buffer per stream (the kernels accumulate into ``.grad``; the
            parameters' grad views are re-pointed before each micro-batch is queued), summed
            into the flat gradient in stream order at the end — deterministic, though not
            the sequential summation order;
          * the BatchNorm running-statistics updates written to per-stream slots, copied to
            a per-micro-batch arena row after each micro-batch and applied in micro-batch
            order once the streams have joined (``UNetEngine.bn_defer_apply``; training-mode
            forwards only write running statistics, so nothing waits for them);
          * its own training meter; the weight-gradient side stream off;
          * stream k replays its own captured micro-batch graph (own static inputs,
            activation pool, gradient buffer and slot; eager for the first GRAPH_WARMUP
            uses) — without graphs the host's ~230 launches per micro-batch are the limit
            once the GPU work overlaps (measured: 93 of a 100 ms step spent enqueueing).
        Parameters do not change inside an accumulation window, so every micro-batch sees
        the same weights as in the one-by-one loop.  The final micro-batch of the window
        runs on the caller's stream as usual (it triggers the gradient exchange)."""
        eng = self.model._engine
        if self.reducer is not None:
            # accumulation micro-batches: no collective (the readiness callbacks of their
            # backwards must not launch bucket all-reduces on a partial gradient)
            self.reducer.prepare(sync=False)
        K = self.micro_streams
        cur = torch.cuda.current_stream(self.device)
        streams = self._ms_streams(K, cur)
        views = self._ms_buffers(K)
        # per-stream graphs by default: without them the host's ~230 launches per
        # micro-batch become the limit once the streams overlap (ms_graph = False: eager)
        use_graph = self.ms_graph
        state = self._ms_enter(K)
        eng.bn_defer_prepare(K, len(mbs))
        order = self.flat.order
        t_host = time.perf_counter()
        for st in streams:
            st.wait_stream(cur)                    # inputs and the previous step are queued
        try:
            for j, (x, y) in enumerate(mbs):
                k = j % K                          # stream k: micro-batches k, k+K, ... in order
                st = streams[k]
                for p, g in zip(order, views[k]):
                    p.grad = g
                eng.bn_defer_j = k
                with torch.cuda.stream(st):
                    if use_graph:
                        self._ms_graph_micro(k, st, x, y)
                    else:
                        self._ms_body(k, x, y)
                    eng.bn_defer_stash(k, j)       # its running-stat slot -> arena row j
                for t in (x, getattr(x, "_ddlpc_nhwc", None), y):
                    if t is not None and t.is_cuda:
                        t.record_stream(st)        # allocated on the caller's stream
        finally:
            self._ms_exit(state)
        self.ms_host_s += time.perf_counter() - t_host     # host enqueue time (diagnostic)
        for st in streams:
            cur.wait_stream(st)
        eng.bn_defer_apply(len(mbs))               # running statistics, in micro-batch order
        self._ms_finish(K, len(mbs))

    def _ms_graph_micro(self, k: int, st, x, y):
        """Stream k's micro-batch as a replay of its own graph (eager for the first
        GRAPH_WARMUP uses, then captured): the batch is copied into stream k's static
        buffers on stream k."""
        from ..data.datasets import engine_input
        xp = getattr(x, "_ddlpc_nhwc", None)
        sk = self._ms_static[k]
        if sk is None or sk[1].shape != y.shape:
            if xp is not None:
                sp = torch.empty_like(xp)
                sk = (engine_input(sp, x.shape[1]), torch.empty_like(y), sp)
            else:
                sk = (torch.empty_like(x), torch.empty_like(y), None)
            self._ms_static[k] = sk
            self._ms_graphs[k], self._ms_warm[k] = None, 0
        sx, sy, sp = sk
        if sp is not None and xp is not None:
            sp.copy_(xp)
        else:
            sx.copy_(x)
        sy.copy_(y)
        g = self._ms_graphs[k]
        if g is not None:
            g.replay()
            return
        self._ms_body(k, sx, sy)
        self._ms_warm[k] += 1
        if self._ms_warm[k] >= self.GRAPH_WARMUP:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                self._ms_body(k, sx, sy)
            self._ms_graphs[k] = g

    # ------------------------------------------------------------------ hipGraph step
    def _graph_ok(self, n_micro: int) -> bool:
        return (self.cfg.hip_graph and self.impl == "hip" and self.device.type == "cuda"
                and not self.cfg.broadcast_buffers and not self.cfg.check_consistency_every
                and (self.reducer is None or n_micro > 1))

    def _static_in(self, x: torch.Tensor, y: torch.Tensor):
        """Copy a micro-batch into the graphs' static input buffers (one pair shared by every
        graph: replays are sequential on one stream).  A device-pipeline batch (padded
        channel-last bf16, ``data.engine_input``) is copied in that layout, so the captured
        forward reads it with no layout pass."""
        from ..data.datasets import engine_input
        xp = getattr(x, "_ddlpc_nhwc", None)
        if self._static is None or self._static[1].shape != y.shape:
            if xp is not None:
                sp = torch.empty_like(xp)
                self._static = (engine_input(sp, x.shape[1]), torch.empty_like(y), sp)
            else:
                self._static = (torch.empty_like(x), torch.empty_like(y), None)
        sx, sy, sp = self._static
        if sp is not None and xp is not None:
            sp.copy_(xp)
        else:
            sx.copy_(x)
        sy.copy_(y)

    def _graph_body(self, kind: str):
        x, y = self._static[0], self._static[1]
        if self.reducer is not None:
            self.reducer.prepare(sync=False)        # "acc": never a collective in a graph
        loss, correct = self.model.loss_and_correct(x, y)
        loss.backward()
        self.meter.add(loss, correct, y.numel())
        if kind == "last":                          # single GPU: the optimizer step too
            self.optimizer.step()
            self.optimizer.zero_grad()

    def _graph_run(self, kind: str):
        """Run one captured micro-batch (``kind`` "acc": forward + backward accumulating into
        the gradient buffer; "last": that + Adam (device-side bias corrections) + zero_grad +
        weight re-pack).  The first ``GRAPH_WARMUP`` calls per kind run eagerly on a side
        stream (allocator + lazy state warm-up); the next eager call is followed by the
        capture (which executes nothing), later calls replay."""
        g = self._graphs.get(kind)
        if g is not None:
            g.replay()
            if kind == "last":
                self.optimizer.note_replayed_step()
            return
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self._graph_body(kind)
        torch.cuda.current_stream(self.device).wait_stream(side)
        self._graph_warm[kind] = self._graph_warm.get(kind, 0) + 1
        if self._graph_warm[kind] >= self.GRAPH_WARMUP:
            self.model._engine.join()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._graph_body(kind)
            if kind == "last":
                self.optimizer.step_count -= 1       # the capture ran step() once in Python
            self._graphs[kind] = g

    def _graph_step(self, micro_batches: List[Tuple[torch.Tensor, torch.Tensor]]):
        """One optimizer step with hipGraph-captured micro-batches (~220 kernel launches per
        micro-batch -> one replay): the reference's regime — batch 1 per GPU, 50
        accumulated micro-batches per exchange (ref.py:685-687,750-766) — is launch-bound.
        Accumulation micro-batches replay the "acc" graph; the last one replays "last"
        (single GPU) or, under data parallelism, runs eagerly so the bucketed collectives
        launch from backward as usual, followed by the exchange and Adam."""
        self.model.train()
        ph = self.phases
        if ph is not None:
            ph.mark("start")
        if self._concurrent_ok(len(micro_batches)):
            # accumulation micro-batches: K streams, each replaying its own graph
            self._concurrent_micros(micro_batches[:-1])
            micro_batches = micro_batches[-1:]
        n = len(micro_batches)
        for i, (x, y) in enumerate(micro_batches):
            last = i == n - 1
            if last and self.reducer is not None:
                self._micro(x, y, sync=True)
                break
            self._static_in(x, y)
            self._graph_run("last" if last else "acc")
            self.micro_count += 1
        if self.reducer is not None:
            if ph is not None:
                ph.mark("fwd_bwd")
            with trace_range("ddlpc.grad_sync"):
                self.reducer.finish()
            if ph is not None:
                ph.mark("comm_wait")
            with trace_range("ddlpc.optimizer"):
                self.optimizer.step()
                self.optimizer.zero_grad()
            if ph is not None:
                ph.mark("optimizer")
        if ph is not None:
            ph.end_step()
        self.step_count += 1
        self.profiler.step()

    GRAPH_WARMUP = 3

    def train_step(self, micro_batches: List[Tuple[torch.Tensor, torch.Tensor]]):
        """One optimizer step over ``len(micro_batches)`` accumulated micro-batches."""
        if self.max_inflight > 0 and self.device.type == "cuda":
            while len(self._inflight) >= self.max_inflight:
                self._inflight.pop(0).synchronize()
        out = self._train_step(micro_batches)
        if self.max_inflight > 0 and self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._inflight.append(ev)
        return out

    # ------------------------------------------------------------------ batched BN-group windows
    WINDOW_PIXELS = 64 * 512 * 512          # auto window: up to 64 512^2 images per pass

    # activation bytes per sample of a grouped pass, per summed conv / BN output element:
    # bf16 y1, a1, y2, a2 are saved (2 B per element of the yardstick) plus ~50% for the
    # backward's transient gradients
    WINDOW_BYTES_PER_ELEM = 3.0

    def _window_size(self, n_micro: int) -> int:
        """Micro-batches per batched pass (0: off).  cfg.bn_window: 0 off, k >= 2 up to k,
        -1 auto = as many as fit WINDOW_PIXELS when micro-batches are small and accumulated
        (the reference's regime: batch 1, 50 micro-batches, ref.py:685-687).

        Auto also requires: every BatchNorm shape supported by the grouped kernels
        (``UNetEngine.bn_groups_supported``), no activation recompute (the grouped pass
        saves y1, a1, y2 per block regardless), and a window whose activations fit in half
        of the memory available to the allocator (measured once per window length)."""
        c = self.cfg
        if n_micro < 2 or self.impl != "hip" or c.bn_window in (0, 1):
            return 0
        key = (n_micro, c.bn_window, c.batch_per_gpu, c.tile, c.recompute)
        cache = self.__dict__.setdefault("_window_cache", {})
        if key in cache:
            return cache[key]
        from ..ops.fused_unet import bn_groups_supported
        if not bn_groups_supported(self.model, c.tile):
            if c.bn_window > 1:
                raise ValueError("bn_window: the grouped BatchNorm kernels do not support this "
                                 "U-Net geometry (bn_window=0 runs the micro-batches one by one)")
            cache[key] = 0
            return 0
        if c.bn_window > 1:
            cache[key] = min(c.bn_window, n_micro)
            return cache[key]
        px = c.batch_per_gpu * c.tile ** c.model.dims
        if px > self.SMALL_MICRO_PIXELS or c.recompute > 0:
            cache[key] = 0
            return 0
        from ..utils.flops import unet_activation_elems_per_sample
        per_micro = (self.WINDOW_BYTES_PER_ELEM * c.batch_per_gpu *
                     unet_activation_elems_per_sample(c.model, c.tile))
        avail = self._allocator_bytes_available()
        fit = n_micro if avail == float("inf") else int(0.5 * avail // max(per_micro, 1.0))
        w = min(n_micro, self.WINDOW_PIXELS // px, fit)
        w = w if w >= 2 else 0
        if self.world > 1:
            # every rank must run the same window (same kernels, same bf16 rounding points,
            # same bucket-readiness order): the smallest fit over the ranks wins
            t = torch.tensor([w], dtype=torch.int64,
                             device=self.device if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            w = int(t.item())
        cache[key] = w
        return cache[key]

    def _allocator_bytes_available(self) -> float:
        """Device memory the caching allocator can still hand out (free + cached unused)."""
        if self.device.type != "cuda" or not torch.cuda.is_available():
            return float("inf")
        free, _total = torch.cuda.mem_get_info(self.device)
        return float(free + torch.cuda.memory_reserved(self.device) -
                     torch.cuda.memory_allocated(self.device))

    @staticmethod
    def _cat_window(mbs: List[Tuple[torch.Tensor, torch.Tensor]]):
        """The window's micro-batches as one batch (engine-layout inputs stay in that layout).
        The micro-batches must have equal shapes: each is one BatchNorm group of batch / G
        samples, and the window's mean loss x G is the sum of the micro-batch losses only
        when every micro-batch has the same pixel count."""
        from ..data.datasets import cat_adjacent, engine_input
        shapes = {(tuple(x.shape), tuple(y.shape)) for x, y in mbs}
        if len(shapes) != 1:
            raise ValueError(f"batched BN window: micro-batches of unequal shapes {sorted(shapes)}")
        # (micro-batches that are back-to-back views of one rendered window — data.split_batch
        # — are joined without a copy)
        xps = [getattr(x, "_ddlpc_nhwc", None) for x, _ in mbs]
        if all(xp is not None for xp in xps):
            x = engine_input(cat_adjacent(xps), mbs[0][0].shape[1])
        else:
            x = cat_adjacent([x for x, _ in mbs])
        return x, cat_adjacent([y for _, y in mbs])

    def _window_step(self, micro_batches: List[Tuple[torch.Tensor, torch.Tensor]], W: int):
        """The accumulation window as batched passes of up to W micro-batches, each micro-batch
        its own BatchNorm group (``UNetEngine.bn_groups``).  The weights do not change inside
        the window and a train-mode BatchNorm normalises over its own micro-batch, so this is
        the computation of the micro-batches one by one (ref.py:750-766) up to the convs'
        summation order: the loss of a pass is the mean over its micro-batches' pixels, so
        its gradient is scaled by the number of micro-batches (the reference sums the
        micro-batch gradients).  Only the last pass arms the gradient exchange."""
        eng = self.model._engine
        n = len(micro_batches)
        chunks = [micro_batches[i:i + W] for i in range(0, n, W)]
        for ci, ch in enumerate(chunks):
            x, y = self._cat_window(ch) if len(ch) > 1 else ch[0]
            if self.reducer is not None:
                self.reducer.prepare(sync=ci == len(chunks) - 1)
            eng.bn_groups = len(ch) if len(ch) > 1 else 0
            try:
                loss, correct = self.model.loss_and_correct(x, y)
                if self.reducer is not None and ci == len(chunks) - 1:
                    self.reducer.mark_backward_start()
                (loss * float(len(ch)) if len(ch) > 1 else loss).backward()
            finally:
                eng.bn_groups = 0
            self.meter.add(loss, correct, y.numel(), n=len(ch))
            self.micro_count += len(ch)

    def _train_step(self, micro_batches: List[Tuple[torch.Tensor, torch.Tensor]]):
        W = self._window_size(len(micro_batches))
        if W and len({tuple(x.shape) for x, _ in micro_batches}) != 1:
            W = 0                        # unequal micro-batches (a short last one): one by one
        if W == 0 and self._graph_ok(len(micro_batches)):
            return self._graph_step(micro_batches)
        self.model.train()
        n = len(micro_batches)
        ph = self.phases
        if ph is not None:
            ph.mark("start")
        with trace_range("ddlpc.fwd_bwd"):
            if W:
                self._window_step(micro_batches, W)
            elif self._concurrent_ok(n):
                self._concurrent_micros(micro_batches[:-1])
                self._micro(*micro_batches[-1], sync=True)
            else:
                for i, (x, y) in enumerate(micro_batches):
                    self._micro(x, y, sync=(i == n - 1))
        if ph is not None:
            ph.mark("fwd_bwd")
        if self.reducer is not None:
            with trace_range("ddlpc.grad_sync"):
                self.reducer.finish()
            if ph is not None:
                ph.mark("comm_wait")          # exposed (non-overlapped) all-reduce time
        with trace_range("ddlpc.optimizer"):
            self.optimizer.step()
            self.optimizer.zero_grad()
        if ph is not None:
            ph.mark("optimizer")
            ph.end_step()
        self.profiler.step()
        if self.cfg.broadcast_buffers:
            broadcast_buffers(self.model)
        self.step_count += 1
        k = self.cfg.check_consistency_every
        if k and self.step_count % k == 0:
            assert_replicas_identical(self.model)

    def choose_schedule(self, micro_batches, steps: int = 3, rounds: int = 2) -> Dict[str, float]:
        """Time ``steps`` optimizer steps with the weight-gradient side stream and without
        it, alternating the two ``rounds`` times and keeping each mode's best round, and
        switch to the faster schedule.  (The first timed slot after warm-up is sometimes
        several times slower than steady state — measured at 1024^2 batch 64: 292 ms in the
        first slot vs 166 ms in a dedicated run — so a single side-then-serial pass could
        pick the wrong mode.)  All ranks agree on the choice (MAX of the per-rank times).
        Performs rounds * 2 * (steps + 1) real steps."""
        eng = self.model._engine if self.impl == "hip" else None
        if eng is None or eng._side_stream is None or self.device.type != "cuda":
            return {}
        times: Dict[bool, List[float]] = {True: [], False: []}
        # caching-allocator free-and-retry events per mode: a schedule that ran the allocator
        # out of memory in any round is not chosen (at 1024^2 x 128 an overlapped round that
        # hit a retry was still fastest by its best round, then every timed step retried:
        # 79 img/s instead of ~400)
        retries: Dict[bool, int] = {True: 0, False: 0}
        for _ in range(rounds):
            for mode in (True, False):
                eng.set_side_stream(mode)
                r0 = torch.cuda.memory_stats(self.device).get("num_alloc_retries", 0)
                self.train_step(micro_batches)
                torch.cuda.synchronize(self.device)
                t0 = time.perf_counter()
                for _ in range(steps):
                    self.train_step(micro_batches)
                torch.cuda.synchronize(self.device)
                dr = torch.cuda.memory_stats(self.device).get("num_alloc_retries", 0) - r0
                t = torch.tensor([time.perf_counter() - t0, float(dr)], dtype=torch.float64,
                                 device=self.device)
                if self.world > 1:
                    dist.all_reduce(t, op=dist.ReduceOp.MAX)
                times[mode].append(float(t[0].item()) / steps)
                retries[mode] += int(t[1].item())
        if retries[True] > 0 and retries[False] == 0:
            best = False
        elif retries[False] > 0 and retries[True] == 0:
            best = True
        else:
            best = min(times[True]) <= min(times[False])
        eng.set_side_stream(best)
        return {"side_stream": best, "side_ms": min(times[True]) * 1e3,
                "serial_ms": min(times[False]) * 1e3,
                "side_rounds_ms": [round(v * 1e3, 3) for v in times[True]],
                "serial_rounds_ms": [round(v * 1e3, 3) for v in times[False]],
                "side_alloc_retries": retries[True], "serial_alloc_retries": retries[False]}

    def fit(self) -> Dict[str, float]:
        c = self.cfg
        self.logger.header(c.batch_per_gpu, self.world, c.accum_steps, c.model.width_divisor)
        last = {}
        t_start = time.perf_counter()
        log_t, log_step = t_start, self.step_count
        prefetch = getattr(self.train_set, "prefetch", None)     # host-streamed datasets
        while self.epoch < c.epochs:
            self.sampler.set_epoch(self.epoch)
            self.meter.reset()
            t_ep = time.perf_counter()
            pending: List[Tuple[torch.Tensor, torch.Tensor]] = []
            # resumed mid-epoch: skip the micro-batches the checkpointed steps consumed
            batches = list(self.sampler.batches(c.batch_per_gpu))[self.epoch_step * c.accum_steps:]
            steps_this_epoch = self.epoch_step
            stopped = False
            for bi, idx in enumerate(batches):
                pending.append(self._to_device(*self.train_set.get(idx)))
                if prefetch is not None and bi + 1 < len(batches):
                    prefetch(batches[bi + 1])     # next batch's H2D copy overlaps this step
                if len(pending) < c.accum_steps:
                    continue
                self.train_step(pending)
                pending = []
                steps_this_epoch += 1
                self.epoch_step = steps_this_epoch
                if c.log_every and self.step_count % c.log_every == 0:
                    m = self.meter.reduce()       # synchronises: phase events are complete
                    now = time.perf_counter()
                    imgs = (self.step_count - log_step) * c.batch_per_gpu * c.accum_steps * self.world
                    rec = {"epoch": self.epoch, "step": self.step_count, **m,
                           "images_per_s": imgs / max(now - log_t, 1e-9),
                           "elapsed_s": now - t_start}
                    if self.phases is not None:
                        rec.update(self.phases.read())
                    log_t, log_step = now, self.step_count
                    self.logger.log(rec)
                if c.ckpt_dir and c.ckpt_every and self.step_count % c.ckpt_every == 0:
                    self.save()
                if (self.rank == c.fault_rank and self.step_count == c.fault_step
                        and os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") == "0"):
                    self.logger.close()
                    mark_dir = c.ckpt_dir or c.log_dir
                    if mark_dir:                  # evidence for tests / post-mortems
                        os.makedirs(mark_dir, exist_ok=True)
                        with open(os.path.join(mark_dir, f"fault_rank{self.rank}_step"
                                               f"{self.step_count}.marker"), "w") as f:
                            f.write("injected\n")
                    os._exit(17)                  # injected fault: this rank dies
                if c.max_steps and self.step_count >= c.max_steps:
                    stopped = bi + 1 < len(batches)
                    break
            if stopped:
                # max_steps inside an epoch: the epoch is NOT finished — keep (epoch,
                # epoch_step) so a resume with a larger max_steps continues right here
                last = self.meter.reduce()
                last.update(epoch=self.epoch, epoch_s=time.perf_counter() - t_ep,
                            steps=self.step_count, partial_epoch=True)
                break
            # leftover micro-batches: gradients stay accumulated into the next epoch's first
            # step, as in the reference (ref.py:748: 127 % 50 = 27 carry over).
            for x, y in pending:
                self._micro(x, y, sync=False)
            ep_s = time.perf_counter() - t_ep
            last = self.meter.reduce()
            last.update(epoch=self.epoch, epoch_s=ep_s, steps=self.step_count)
            self.logger.epoch_line(self.epoch, last["loss"], last["pixel_acc"], ep_s,
                                   ep_s / max(steps_this_epoch, 1))
            self.logger.log({"epoch_end": self.epoch, **last})
            if c.png_dir and self.rank == 0:
                x, y = self.train_set.get(list(range(min(c.png_count, len(self.train_set)))))
                dump_pngs(self.model, *self._to_device(x, y), c.png_dir, c.png_count)
            self.epoch += 1
            self.epoch_step = 0
            if c.max_steps and self.step_count >= c.max_steps:
                break
        if c.ckpt_dir:
            self.save()
        return last

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def validate(self, dataset=None, batch: Optional[int] = None) -> Dict[str, float]:
        """Held-out loss, pixel accuracy and per-class IoU (the reference never evaluates its
        30-tile test split, ref.py:672-673), sharded over ranks and all-reduced."""
        ds = dataset if dataset is not None else self.test_set
        if ds is None or len(ds) == 0:
            return {}
        self.model.eval()
        k = self.cfg.model.out_classes
        bs = batch or self.cfg.batch_per_gpu
        acc = torch.zeros(3, dtype=torch.float64, device=self.device)
        cm = torch.zeros(k * k, dtype=torch.float64, device=self.device)
        idx_all = list(range(len(ds)))[self.rank::self.world]
        for i in range(0, len(idx_all), bs):
            x, y = self._to_device(*ds.get(idx_all[i:i + bs]))
            ctx = (torch.autocast("cuda", dtype=torch.bfloat16) if self.autocast
                   else contextlib.nullcontext())
            with ctx:
                logits = self.model(x)
            logits = logits.float()
            loss = torch.nn.functional.cross_entropy(logits, y, reduction="sum")
            pred = logits.argmax(1)
            acc += torch.stack([loss.double(), (pred == y).sum().double(),
                                torch.tensor(float(y.numel()), device=self.device,
                                             dtype=torch.float64)])
            cm += torch.bincount((y * k + pred).reshape(-1), minlength=k * k).double()
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(acc)
            dist.all_reduce(cm)
        self.model.train()
        cmm = cm.reshape(k, k)
        inter = cmm.diag()
        union = cmm.sum(0) + cmm.sum(1) - inter
        iou = (inter / union.clamp_min(1)).tolist()
        valid = (union > 0).tolist()
        miou = [v for v, ok in zip(iou, valid) if ok]
        a = acc.tolist()
        return {"val_loss": a[0] / max(a[2], 1), "val_pixel_acc": a[1] / max(a[2], 1),
                "val_iou": iou, "val_miou": sum(miou) / max(len(miou), 1)}

    # ------------------------------------------------------------------ checkpoint
    def save(self, path: Optional[str] = None) -> Optional[str]:
        path = path or os.path.join(self.cfg.ckpt_dir, f"ckpt_{self.step_count}.pt")
        if self.rank == 0:
            save_checkpoint(path, self.model, self.optimizer, epoch=self.epoch,
                            step=self.step_count, micro_step=self.micro_count,
                            config=self.cfg.to_dict(), epoch_step=self.epoch_step)
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
        return path

    def load(self, path: str):
        blob = load_checkpoint(path, self.model, self.optimizer)
        self.epoch = int(blob.get("epoch", 0))
        self.step_count = int(blob.get("step", 0))
        self.micro_count = int(blob.get("micro_step", 0))
        self.epoch_step = int(blob.get("epoch_step", 0))
        if self.model._engine is not None:
            self.model._engine.pack_weights()
        return blob

    def close(self):
        self.profiler.close()
        self.logger.close()
        if self.reducer is not None:
            self.reducer.remove_hooks()


class _Subset:
    def __init__(self, base, start, end):
        self.base, self.start, self.end = base, start, end

    def __len__(self):
        return self.end - self.start

    @property
    def on_device(self) -> bool:
        return getattr(self.base, "on_device", False)

    def get(self, idx):
        if torch.is_tensor(idx):         # device indices stay on the device (no host sync)
            return self.base.get(idx.reshape(-1).to(torch.int64) + self.start)
        return self.base.get([self.start + int(i) for i in idx])


def train(cfg: TrainConfig, device: Optional[str] = None, return_trainer: bool = False):
    """Train per ``cfg``; returns the last epoch's reduced metrics (and the trainer)."""
    tr = Trainer(cfg, device)
    try:
        m = tr.fit()
    finally:
        tr.close()
    return (m, tr) if return_trainer else m


def validate(cfg_or_trainer, checkpoint: Optional[str] = None,
             device: Optional[str] = None) -> Dict[str, float]:
    """Evaluate a trainer, or build one from ``cfg`` (+ optional checkpoint) and evaluate."""
    if isinstance(cfg_or_trainer, Trainer):
        return cfg_or_trainer.validate()
    tr = Trainer(cfg_or_trainer, device)
    if checkpoint:
        tr.load(checkpoint)
    try:
        return tr.validate()
    finally:
        tr.close()
