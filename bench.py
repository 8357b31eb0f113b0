#!/usr/bin/env python
"""Headline benchmark: whole-node training images/sec, U-Net 5-level, 256x256, 6 classes.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` — for N>1 launched by
``torch.distributed.run`` with one rank per GPU (RCCL).  W untimed warm-up steps, then
exactly K timed optimizer steps bracketed by barrier + device synchronize on both sides;
the per-rank time is MAX-reduced and rank 0 prints ONE JSON line.  ``value`` is the
aggregate images/sec over all N GPUs (weak scaling: fixed per-GPU batch).

``--gpus N`` with N > 1 outside torchrun spawns torchrun itself (child process, before
anything touches the GPU); a torchrun ``WORLD_SIZE`` that disagrees with ``--gpus`` is an
error (exit 2) — a mis-launched run never publishes a 1-GPU number as an N-GPU one.

Model/config (BASELINE.json): the reference U-Net (ref.py:620-656) with its shipped width
divisor 2 (8.72 M params), 5 levels, conv-transpose up-sampling, 6 classes, 256x256 RGB
synthetic Vaihingen-shape tiles, random-init weights, bf16 compute with fp32 master
weights, CrossEntropy + Adam (ref.py:703-704).  Inside the timed region every step
renders its batch in HBM (the trainer's own device input pipeline, ``synth_tiles``
kernel, distinct sample indices per rank and step), then runs the full forward +
backward + gradient all-reduce + optimizer step.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (images); default 384 for the flagship 256^2 2-D config "
                         "(same box: 256 / 384 / 512 -> 7838 / 7985 / 7967 img/s, 30 GB of the "
                         "288 GB HBM; profiles/r6/batch_sweep_r6b_*), 128 otherwise; "
                         "32 / 64 / 128 / 256 / 384 have measured in-house baselines")
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--tile", type=int, default=256)
    ap.add_argument("--width-divisor", type=int, default=2)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--classes", type=int, default=6)
    ap.add_argument("--dims", type=int, default=2, help="2 = images, 3 = volumes (3-D U-Net)")
    ap.add_argument("--impl", default=os.environ.get("DDLPC_IMPL", "hip"),
                    choices=["hip", "torch"])
    ap.add_argument("--bucket-mb", type=float, default=8.0,
                    help="largest gradient bucket (fp32 MB)")
    ap.add_argument("--bucket-plan", default="readiness", choices=["readiness", "size"],
                    help="readiness: cuts from the backward readiness model "
                         "(parallel/bucket_plan.py); size: cut by size only")
    ap.add_argument("--bucket-sweep", default="",
                    help="comma list of bucket sizes (MB) timed after the main run (N>1), "
                         "e.g. 2,4,8,16,35; reported as config.bucket_sweep")
    ap.add_argument("--wire-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--codec", default="none")
    ap.add_argument("--verbose", type=int, default=0, help="1: progress lines on stderr")
    ap.add_argument("--schedule", default="auto", choices=["auto", "overlap", "serial"],
                    help="weight-gradient stream: auto = time both during warm-up, keep the faster")
    ap.add_argument("--hip-graph", type=int, default=int(os.environ.get("DDLPC_HIP_GRAPH", "0")),
                    help="1: replay the single-GPU train step as one hipGraph")
    ap.add_argument("--recompute", type=int, default=0,
                    help="activation recompute in backward: 1 = first conv of each block, "
                         "2 = both convs (less activation memory, more compute)")
    ap.add_argument("--fixed-batch", type=int, default=0,
                    help="diagnostic: 1 = reuse one rendered batch every step (no per-step "
                         "input pipeline; reported in 'data')")
    ap.add_argument("--micro-streams", type=int, default=-1,
                    help="accumulation micro-batches in flight on this many HIP streams "
                         "(-1: auto, 3 for small accumulated micro-batches)")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="CUs kept out of persistent kernel grids (-1: auto = 0, measured: "
                         "see docs/PERF.md 'Data-parallel overlap')")
    ap.add_argument("--comm-proxy", type=int, default=0,
                    help="1 GPU: stand-in collective per gradient bucket for a world of N "
                         "(streaming kernel on a third stream; measures launch-to-finish "
                         "latency during backward)")
    ap.add_argument("--prefetch", type=int, default=0,
                    help="1: render the next step's on-device batch on a side stream under "
                         "this step (0, default: in front of each step; same box 7980 / 7994 "
                         "vs 7994 / 8017 img/s — the generator shares HBM with the step either "
                         "way: profiles/r6/prefetch_proxy_r6i_*)")
    ap.add_argument("--engine-set", default="",
                    help="diagnostic: NAME=INT[,NAME=INT] — set UNetEngine switches (e.g. "
                         "c32_bnp=0) before the first step, for same-box A/B runs")
    ap.add_argument("--ab", default="",
                    help="diagnostic: KNOB:v0,v1 — after the main timing, alternate a kernel "
                         "knob over --ab-rounds timed blocks in this process; reported as "
                         "config.ab.  CU_RESERVE = set_cu_reserve; any other name must be a "
                         "knob a kernel reads (csrc/bindings.cpp kKnobs), else set_knob "
                         "raises before anything is timed")
    ap.add_argument("--ab-rounds", type=int, default=4)
    ap.add_argument("--heartbeat", type=float, default=0.0,
                    help="seconds between 'alive' lines on stderr (long first-step autotuning)")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = 384 if (a.tile == 256 and a.dims == 2) else 128
    return a


def _launch_guard(args) -> None:
    """Enforce the one-rank-per-GPU contract BEFORE any GPU call."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus > 1:
            # not under torchrun: become the launcher (a child process, never an exec)
            # (c10d rendezvous on port 0: the agent's store binds its own port, no race)
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={args.gpus}", "--rdzv-backend=c10d",
                   "--rdzv-endpoint=127.0.0.1:0", os.path.abspath(__file__)] + sys.argv[1:]
            print(f"bench: spawning {args.gpus} ranks via torchrun", file=sys.stderr, flush=True)
            sys.exit(subprocess.call(cmd))
        return
    if int(ws) != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={ws}: refusing to report a "
              f"{ws}-rank number as {args.gpus}-GPU", file=sys.stderr, flush=True)
        sys.exit(2)


def _baseline(args):
    """In-house MIOpen baseline (BASELINE.json) for the SAME config, else None."""
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            b = json.load(f).get("inhouse_baseline", {})
    except Exception:
        return None
    if args.accum != 1 or args.classes != 6 or args.depth != 5:
        return None
    if args.dims == 3:
        # no meaningful 3-D anchor: the only stock run (0.59 vol/s) needed MIOpen's FAST find
        # mode because the exhaustive search did not finish (BASELINE.json d3_128_note)
        return None
    if args.tile != 256:
        return None
    if args.width_divisor == 1:
        v = b.get("wd1_images_per_sec", {}).get(str(args.batch))
        return float(v) if v else None
    if args.width_divisor != 2:
        return None
    v = {32: b.get("images_per_sec_per_gpu"), 64: b.get("batch_64_images_per_sec"),
         128: b.get("batch_128_images_per_sec"), 256: b.get("batch_256_images_per_sec"),
         384: b.get("batch_384_images_per_sec")}.get(args.batch)
    return float(v) if v else None


def main():
    args = _parse()
    _launch_guard(args)
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    if args.heartbeat > 0:
        import threading

        def _beat():
            t0 = time.time()
            while True:
                time.sleep(args.heartbeat)
                print(f"alive {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
        threading.Thread(target=_beat, daemon=True).start()

    from ddlpc.config import ModelConfig, TrainConfig
    from ddlpc.data import device_random_batch
    from ddlpc.train.trainer import Trainer

    cfg = TrainConfig(model=ModelConfig(out_classes=args.classes, depth=args.depth,
                                        width_divisor=args.width_divisor, dims=args.dims),
                      tile=args.tile, batch_per_gpu=args.batch, accum_steps=args.accum,
                      num_samples=1 << 30, test_holdout=0, impl=args.impl,
                      bucket_mb=args.bucket_mb, bucket_plan=args.bucket_plan,
                      wire_dtype=args.wire_dtype,
                      grad_codec=args.codec, log_dir=None, hip_graph=bool(args.hip_graph),
                      recompute=int(args.recompute), reserve_cus=args.reserve_cus,
                      comm_proxy=args.comm_proxy, micro_streams=args.micro_streams)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    tr = Trainer(cfg, device=dev)
    if args.engine_set and tr.impl == "hip":
        eng = tr.model._engine
        for kv in args.engine_set.split(","):
            k, v = kv.split("=")
            if not hasattr(eng, k) or isinstance(getattr(eng, k), torch.Tensor):
                raise SystemExit(f"--engine-set: UNetEngine has no switch {k!r}")
            setattr(eng, k, type(getattr(eng, k))(int(v)))
    world, rank = tr.world, tr.rank
    assert world == args.gpus, (world, args.gpus)
    device = tr.device
    B = args.batch
    on_device_data = tr.impl == "hip"     # (rendered by the synth_tiles op, GPU or CPU kernel)
    pool = []
    if not on_device_data:
        # stock-op baseline / CPU: a small pre-rendered pool (the baseline's published
        # numbers were measured this way)
        for i in range(4):
            x, y = device_random_batch(B, args.tile, args.classes, device,
                                       seed=1000 * rank + i, dims=args.dims,
                                       dtype=torch.bfloat16 if dev == "cuda" else torch.float32,
                                       channels_last=(dev == "cuda"))
            if dev == "cpu":
                x = x.float()
            pool.append((x, y))

    def batch(k):
        if on_device_data:
            # global micro-batch k, this rank's slice of distinct sample indices
            start = (k * world + rank) * B
            idx = torch.arange(start, start + B, device=device, dtype=torch.int64)
            return tr.train_set.get(idx)
        return pool[k % len(pool)]

    def window(i):
        # on-device data: the step's accum micro-batches rendered in ONE pass (one index
        # vector, one synth launch) and handed out as zero-copy views (data.split_batch; the
        # batched BN window joins them back without a copy); each micro-batch holds the same
        # distinct samples as micro-batch-by-micro-batch rendering would
        if on_device_data and args.accum > 1:
            from ddlpc.data import split_batch
            ks = torch.arange(i * args.accum, (i + 1) * args.accum, device=device, dtype=torch.int64)
            idx = ((ks * world + rank) * B)[:, None] + torch.arange(B, device=device, dtype=torch.int64)
            return split_batch(*tr.train_set.get(idx.reshape(-1)), args.accum)
        return [batch(i * args.accum + j) for j in range(args.accum)]

    fixed = window(0) if args.fixed_batch else None
    # on-device data: step i+1's batch renders on a side stream under step i (one batch per
    # step is still rendered inside the timed region; data.DevicePrefetcher)
    pf = None
    if on_device_data and fixed is None and args.prefetch:
        from ddlpc.data import DevicePrefetcher
        pf = DevicePrefetcher(window, device)

    def step(i):
        tr.train_step(fixed if fixed is not None else pf.get(i) if pf is not None else window(i))

    def sync():
        if dev == "cuda":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        if dev == "cuda":
            torch.cuda.synchronize()

    def timed(n, first):
        sync()
        t0 = time.perf_counter()
        for i in range(n):
            step(first + i)
        sync()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for i in range(args.warmup):
        step(i)
        if args.verbose and rank == 0:
            print(f"warmup step {i} done", file=sys.stderr, flush=True)
    # schedule calibration (untimed): overlapped weight-gradient stream vs serial
    sched = {}
    if args.schedule == "auto":
        sched = tr.choose_schedule(window(10_000))
        if rank == 0 and sched:
            print(f"schedule: {sched}", file=sys.stderr, flush=True)
    elif args.schedule == "serial" and tr.impl == "hip":
        tr.model._engine.set_side_stream(False)
    # readiness-aware buckets re-planned from one measured step (untimed): every gradient's
    # ready time and the backward time instead of the FLOP-rate model (all ranks cut alike)
    calib = tr.calibrate_bucket_plan(window(20_000)) if tr.reducer is not None else None
    if tr.phases is not None:
        tr.phases.read(reset=True)                 # phase means over the timed steps only
    first = args.warmup + 100
    tr.ms_host_s = 0.0
    dt = timed(args.steps, first)
    phases = tr.phases.read() if tr.phases is not None else {}
    ms_host = getattr(tr, "ms_host_s", 0.0)
    mstats = torch.cuda.memory_stats(device) if dev == "cuda" else {}
    ms = dt / args.steps * 1e3
    imgs = B * args.accum * world * args.steps
    value = imgs / dt
    sweep = {}
    if args.bucket_sweep and world > 1:
        for mb in [float(v) for v in args.bucket_sweep.split(",") if v]:
            nb = tr.set_bucket_mb(mb)
            first += args.steps + 2
            step(first - 1)                        # one untimed step at the new size
            sweep[str(mb)] = {"buckets": nb,
                              "ms_per_step": round(timed(args.steps, first) / args.steps * 1e3, 3)}
        tr.set_bucket_mb(args.bucket_mb)
    ab = None
    if args.ab and tr.impl == "hip":
        from ddlpc.ops import _ext
        F = _ext.ops()
        knob, vals = args.ab.split(":")
        vals = [int(v) for v in vals.split(",")]

        prev = []

        def setk(v):
            if knob == "CU_RESERVE":
                F.set_cu_reserve(v)
            else:
                p = F.set_knob(knob, v)
                if not prev:
                    prev.append(p)                     # the value before the A/B
        ab = {str(v): [] for v in vals}
        for r in range(args.ab_rounds):
            for v in vals:
                setk(v)
                first += args.steps + 2
                step(first - 1)                        # one untimed step with the new setting
                ab[str(v)].append(round(timed(args.steps, first) / args.steps * 1e3, 3))
        # restore the pre-A/B state (INT64_MIN clears the override: environment / default)
        if knob == "CU_RESERVE":
            F.set_cu_reserve(tr.reserve_cus)
        elif prev:
            F.set_knob(knob, prev[0])
        # (per-round ratios against the first value cancel clock / thermal drifts across rounds)
        v0 = str(vals[0])
        paired = {v: sorted(a / b for a, b in zip(x, ab[v0]))[len(x) // 2] for v, x in ab.items()}
        ab = {"knob": knob, "ms_per_step": ab,
              "median_ms": {v: sorted(x)[len(x) // 2] for v, x in ab.items()},
              "median_paired_ratio": {v: round(r, 4) for v, r in paired.items()}}
    proxy = None
    if tr.reducer is not None and tr.reducer.proxy:
        proxy = [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}
                 for d in tr.reducer.proxy_times()]
        plan = getattr(tr, "bucket_plan", None)
        if plan is not None and len(plan.bucket_done_ms) == len(proxy):
            # the plan's predicted end of every bucket's collective against the proxy's
            # measured end (both from the backward start of the last timed step)
            for rec, pred in zip(proxy, plan.bucket_done_ms):
                rec["predicted_end_ms"] = round(pred, 3)
                if "end_from_backward_start_ms" in rec:
                    rec["predicted_minus_measured_ms"] = round(pred - rec["end_from_backward_start_ms"], 3)
    # self-validation of a multi-rank run (after the timed steps, untimed): the backend and
    # world the collectives really ran on, and bit-identical replicas (every rank applied the
    # same reduced gradient); a diverged run still prints its line but exits non-zero
    dist_rec = {"dist_backend": None, "world_size": 1, "rccl_version": None,
                "replicas_identical": None}
    diverged = False
    if world > 1:
        from ddlpc.parallel import assert_replicas_identical
        dist_rec["dist_backend"] = str(dist.get_backend())
        dist_rec["world_size"] = dist.get_world_size()
        if dist_rec["dist_backend"] == "nccl":
            try:
                v = torch.cuda.nccl.version()
                dist_rec["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
            except Exception as e:  # noqa: BLE001
                dist_rec["rccl_version"] = f"unknown ({type(e).__name__})"
        try:
            assert_replicas_identical(tr.model)
            dist_rec["replicas_identical"] = True
        except RuntimeError as e:
            dist_rec["replicas_identical"] = False
            diverged = True
            print(f"bench: {e}", file=sys.stderr, flush=True)
        if dist_rec["world_size"] != args.gpus:
            diverged = True
    base = _baseline(args)
    from ddlpc.utils.flops import PEAK_BF16_TFLOPS, unet_train_flops_per_sample
    flop_img = unet_train_flops_per_sample(cfg.model, args.tile)
    tflops = value * flop_img / 1e12                     # whole job
    loss = tr.meter.reduce()
    if args.dims == 2:
        metric = f"images/sec (whole node), U-Net {args.tile}x{args.tile} {args.classes}-class tiles"
        data_desc = (f"synthetic (Vaihingen-shape {args.tile}x{args.tile} RGB tiles rendered in HBM "
                     f"per step, {args.classes} classes, random-init weights)")
    else:
        metric = (f"volumes/sec (whole node), 3-D U-Net {args.tile}^3 {args.classes}-class volumes")
        data_desc = (f"synthetic ({args.tile}^3 3-channel volumes rendered in HBM per step, "
                     f"{args.classes} classes, random-init weights)")
    if not on_device_data:
        data_desc = data_desc.replace("rendered in HBM per step", "pre-rendered pool of 4 batches")
    elif args.fixed_batch:
        data_desc = data_desc.replace("rendered in HBM per step", "ONE batch rendered once (diagnostic)")
    elif pf is not None:
        data_desc = data_desc.replace("rendered in HBM per step",
                                      "rendered in HBM per step, one step ahead on a side stream")
    if rank == 0:
        red = tr.reducer
        rec = {
            "metric": metric,
            "value": round(value, 2), "unit": "images/s" if args.dims == 2 else "volumes/s",
            "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (round(value / (base * world), 3) if base else None),
            # roofline: model-geometry FLOPs (3 x forward conv MACs x 2, utils/flops.py) per
            # second, and that as a fraction of world x 2.5 PF dense bf16
            "tflops_per_s": round(tflops, 1),
            "mfu": round(tflops / (PEAK_BF16_TFLOPS * world), 4),
            "gflop_per_sample": round(flop_img / 1e9, 2),
            # compute dtype: the engine (either device) and GPU autocast run bf16; the stock
            # modules on a CPU run fp32
            "dtype": "bf16" if (tr.impl == "hip" or dev == "cuda") else "fp32",
            "data": data_desc,
            **dist_rec,
            "comm_wait_ms": (round(phases["comm_wait_ms"], 3) if "comm_wait_ms" in phases
                             else None),
            "config": {"model": f"UNet depth{args.depth} width/{args.width_divisor} "
                                f"conv_transpose ({sum(p.numel() for p in tr.model.parameters())} params)",
                       "global_batch": B * args.accum * world,
                       "per_gpu_batch": B, "accum_steps": args.accum,
                       "seq_len": None, "tile": args.tile, "dims": args.dims,
                       "classes": args.classes,
                       "parallelism": f"dp{world}" + (f"+comm_proxy{args.comm_proxy}"
                                                       if args.comm_proxy else ""),
                       "impl": tr.impl,
                       "reserve_cus": getattr(tr, "reserve_cus", None),
                       "comm_proxy_last_step": proxy,
                       "optimizer": "Adam(lr=1e-3)", "loss": "CrossEntropy",
                       "train_loss_mean": round(loss["loss"], 4),
                       "recompute": int(args.recompute),
                       "micro_streams": getattr(tr, "micro_streams", 1),
                       # accumulation micro-batches per batched pass with per-micro-batch
                       # BatchNorm groups (0: off; the micro_streams schedule then applies)
                       "bn_window": (tr._window_size(args.accum) if hasattr(tr, "_window_size")
                                     else 0),
                       "micro_streams_host_ms_per_step": (round(ms_host * 1e3 / args.steps, 2)
                                                          if getattr(tr, "micro_streams", 1) > 1
                                                          else None),
                       "peak_mem_gb": (round(torch.cuda.max_memory_allocated(device) / 2**30, 2)
                                       if dev == "cuda" else None),
                       "schedule": ("overlap" if sched.get("side_stream") else "serial") if sched
                                   else args.schedule,
                       "schedule_probe_ms": ({k: (round(v, 3) if isinstance(v, float) else v)
                                              for k, v in sched.items() if k.endswith("_ms")}
                                             if sched else None),
                       "schedule_probe_alloc_retries": ({k: v for k, v in sched.items()
                                                         if k.endswith("_alloc_retries")}
                                                        if sched else None),
                       "bucket_mb": args.bucket_mb,
                       "buckets": len(red.buckets) if red is not None else 0,
                       "bucket_plan": cfg.bucket_plan,
                       "bucket_sizes_mb": ([round((b.end - b.start) * 4 / 2**20, 3)
                                            for b in red.buckets] if red is not None else None),
                       "bucket_plan_calibration": calib,
                       "bucket_plan_predicted_exposed_ms": (
                           round(tr.bucket_plan.exposed_ms, 3)
                           if getattr(tr, "bucket_plan", None) is not None else None),
                       "wire_dtype": args.wire_dtype, "grad_codec": args.codec,
                       "phase_ms": {k: round(v, 3) for k, v in phases.items()},
                       "comm_wait_ms": (round(phases["comm_wait_ms"], 3)
                                        if "comm_wait_ms" in phases else None),
                       "bucket_sweep": sweep or None,
                       "ab": ab,
                       "engine_set": args.engine_set or None,
                       "input_prefetch": pf is not None,
                       "alloc_retries": mstats.get("num_alloc_retries"),
                       "side_lag_waits": (getattr(tr.model._engine, "lag_waits", None)
                                          if tr.impl == "hip" else None),
                       "device_mallocs": mstats.get("num_device_alloc"),
                       "device_frees": mstats.get("num_device_free")},
        }
        print(json.dumps(rec), flush=True)
    tr.close()
    if world > 1:
        dist.destroy_process_group()
    if diverged:
        sys.exit(3)


if __name__ == "__main__":
    main()
