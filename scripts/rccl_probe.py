#!/usr/bin/env python
"""Probe: can two ranks run RCCL (`nccl` backend) collectives when they share ONE GPU?

    python scripts/rccl_probe.py [--world 2] [--mb 64]

Spawns `world` processes on cuda:0 (127.0.0.1 rendezvous), all-reduces a `mb`-MiB bf16/fp32
buffer a few times and checks the sum.  RCCL normally rejects two ranks on one device
("Duplicate GPU detected"); the outcome is printed either way, one line per rank.
"""
import argparse
import os
import sys
import time


def _worker(rank, world, port, mb, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
        n = mb * (1 << 20) // 4
        x = torch.full((n,), float(rank + 1), device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        want = world * (world + 1) / 2
        ok = bool((x == want).all().item())
        t0 = time.time()
        for _ in range(5):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / 5
        q.put((rank, "ok" if ok else "WRONG SUM", f"{mb} MiB all-reduce {dt * 1e3:.2f} ms"))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - report whatever RCCL says
        q.put((rank, "error", repr(e)[:400]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mb", type=int, default=64)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29611
    ps = [ctx.Process(target=_worker, args=(r, a.world, port, a.mb, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = []
    for _ in ps:
        try:
            res.append(q.get(timeout=90))
        except Exception:  # noqa: BLE001
            res.append((-1, "timeout", "no answer within 90 s"))
    for p in ps:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
    for r in sorted(res):
        print("rank", *r, flush=True)
    return 0 if all(r[1] == "ok" for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
