#!/usr/bin/env python
"""Headline benchmark: whole-node training images/sec, U-Net 5-level, 256x256, 6 classes.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` — for N>1 launched by
``torch.distributed.run`` with one rank per GPU (RCCL).  W untimed warm-up steps, then
exactly K timed optimizer steps bracketed by barrier + device synchronize on both sides;
the per-rank time is MAX-reduced and rank 0 prints ONE JSON line.  ``value`` is the
aggregate images/sec over all N GPUs (weak scaling: fixed per-GPU batch).

Model/config (BASELINE.json): the reference U-Net (ref.py:620-656) with its shipped width
divisor 2 (8.72 M params), 5 levels, conv-transpose up-sampling, 6 classes, 256x256 RGB
synthetic Vaihingen-shape tiles, random-init weights, bf16 compute with fp32 master
weights, CrossEntropy + Adam (ref.py:703-704), full forward + backward + gradient
all-reduce + optimizer step inside the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_IMG_S = None   # set from BASELINE.json "inhouse_baseline" if present


def _baseline(args):
    """In-house MIOpen baseline (BASELINE.json) for the SAME config, else None."""
    if args.dims != 2 or args.tile != 256 or args.depth != 5 or args.width_divisor != 2 \
            or args.classes != 6 or args.accum != 1:
        return None
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "BASELINE.json")
    try:
        with open(p) as f:
            b = json.load(f).get("inhouse_baseline", {})
        v = {32: b.get("images_per_sec_per_gpu"), 64: b.get("batch_64_images_per_sec"),
             128: b.get("batch_128_images_per_sec")}.get(args.batch)
        return float(v) if v else None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128,
                    help="per-GPU batch (images); 32 / 64 / 128 have measured in-house baselines")
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--tile", type=int, default=256)
    ap.add_argument("--width-divisor", type=int, default=2)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--classes", type=int, default=6)
    ap.add_argument("--dims", type=int, default=2, help="2 = images, 3 = volumes (3-D U-Net)")
    ap.add_argument("--impl", default=os.environ.get("DDLPC_IMPL", "hip"),
                    choices=["hip", "torch"])
    ap.add_argument("--bucket-mb", type=float, default=8.0)
    ap.add_argument("--codec", default="none")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--verbose", type=int, default=0, help="1: progress lines on stderr")
    ap.add_argument("--schedule", default="auto", choices=["auto", "overlap", "serial"],
                    help="weight-gradient stream: auto = time both during warm-up, keep the faster")
    ap.add_argument("--hip-graph", type=int, default=int(os.environ.get("DDLPC_HIP_GRAPH", "0")),
                    help="1: replay the single-GPU train step as one hipGraph")
    ap.add_argument("--heartbeat", type=float, default=0.0,
                    help="seconds between 'alive' lines on stderr (long first-step autotuning)")
    args = ap.parse_args()
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
                      num_samples=1, test_holdout=0, impl=args.impl, bucket_mb=args.bucket_mb,
                      grad_codec=args.codec, log_dir=None, hip_graph=bool(args.hip_graph))
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    tr = Trainer(cfg, device=dev)
    world, rank = tr.world, tr.rank
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    device = tr.device
    # a small pool of distinct device-resident batches (synthetic; no host I/O in the loop)
    pool = []
    for i in range(4):
        x, y = device_random_batch(args.batch, args.tile, args.classes, device,
                                   seed=1000 * rank + i, dims=args.dims,
                                   dtype=torch.bfloat16 if dev == "cuda" else torch.float32,
                                   channels_last=(dev == "cuda"))
        if tr.impl == "torch":
            x = x.float() if dev == "cpu" else x
        pool.append((x, y))

    def step(i):
        mbs = [pool[(i * args.accum + j) % len(pool)] for j in range(args.accum)]
        tr.train_step(mbs)

    def sync():
        if dev == "cuda":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        if dev == "cuda":
            torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
        if args.verbose and rank == 0:
            print(f"warmup step {i} done", file=sys.stderr, flush=True)
    # schedule calibration (untimed): overlapped weight-gradient stream vs serial
    sched = {}
    if args.schedule == "auto":
        sched = tr.choose_schedule(pool[0:1] if args.accum == 1 else
                                   [pool[j % len(pool)] for j in range(args.accum)])
        if rank == 0 and sched:
            print(f"schedule: {sched}", file=sys.stderr, flush=True)
    elif args.schedule == "serial" and tr.impl == "hip":
        tr.model._engine.set_side_stream(False)
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    sync()
    dt = time.perf_counter() - t0
    mstats = torch.cuda.memory_stats(device) if dev == "cuda" else {}
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1e3
    imgs = args.batch * args.accum * world * args.steps
    value = imgs / dt
    base = _baseline(args)
    loss = tr.meter.reduce()
    if args.dims == 2:
        metric = f"images/sec (whole node), U-Net {args.tile}x{args.tile} {args.classes}-class tiles"
        data_desc = (f"synthetic (Vaihingen-shape {args.tile}x{args.tile} RGB tiles, "
                     f"{args.classes} classes, random-init weights)")
    else:
        metric = (f"volumes/sec (whole node), 3-D U-Net {args.tile}^3 {args.classes}-class volumes")
        data_desc = (f"synthetic ({args.tile}^3 3-channel volumes, {args.classes} classes, "
                     "random-init weights)")
    if rank == 0:
        rec = {
            "metric": metric,
            "value": round(value, 2), "unit": "images/s" if args.dims == 2 else "volumes/s",
            "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (round(value / (base * world), 3) if base else None),
            "dtype": "bf16" if dev == "cuda" else "fp32",
            "data": data_desc,
            "config": {"model": f"UNet depth{args.depth} width/{args.width_divisor} "
                                f"conv_transpose ({sum(p.numel() for p in tr.model.parameters())} params)",
                       "global_batch": args.batch * args.accum * world,
                       "per_gpu_batch": args.batch, "accum_steps": args.accum,
                       "seq_len": None, "tile": args.tile, "dims": args.dims,
                       "classes": args.classes,
                       "parallelism": f"dp{world}", "impl": tr.impl,
                       "optimizer": "Adam(lr=1e-3)", "loss": "CrossEntropy",
                       "train_loss_mean": round(loss["loss"], 4),
                       "peak_mem_gb": (round(torch.cuda.max_memory_allocated(device) / 2**30, 2)
                                       if dev == "cuda" else None),
                       "schedule": ("overlap" if sched.get("side_stream") else "serial") if sched
                                   else args.schedule,
                       "alloc_retries": mstats.get("num_alloc_retries"),
                       "device_mallocs": mstats.get("num_device_alloc"),
                       "device_frees": mstats.get("num_device_free")},
        }
        print(json.dumps(rec), flush=True)
    tr.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
