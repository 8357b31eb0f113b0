"""Spawn a gloo "fake cluster" on localhost (the reference needs 6 named PCs;
this runs the same data-parallel protocol in W processes on 127.0.0.1)."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    os.environ.setdefault("OMP_NUM_THREADS", "2")
    import torch
    torch.set_num_threads(2)
    try:
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, "err", f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


# rendezvous / socket failures of the local gloo mesh (a free_port() race with another
# process, a connect that lost the race): the run is repeated once on a fresh port
_TRANSIENT = ("Address already in use", "Connection refused", "Connection reset",
              "Socket Timeout", "EADDRINUSE", "ECONNREFUSED", "ECONNRESET")


def run(fn, world=2, args=(), timeout=240, allow_fail=False):
    out = _run_once(fn, world, args, timeout)
    if not allow_fail and any(st != "ok" and any(t in str(res) for t in _TRANSIENT)
                              for st, res in out.values()):
        out = _run_once(fn, world, args, timeout)
    if not allow_fail:
        for r, (st, res) in sorted(out.items()):
            assert st == "ok", f"rank {r} failed: {res}"
        assert len(out) == world, f"only {len(out)} of {world} ranks reported"
        return {r: res for r, (st, res) in out.items()}
    return out


def _run_once(fn, world, args, timeout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    import queue as _q
    import time
    t0 = time.time()
    while len(out) < world and time.time() - t0 < timeout:
        try:
            r, status, res = q.get(timeout=1.0)
            out[r] = (status, res)
        except _q.Empty:
            # a rank that died without reporting (fault injection) never will
            if all(not p.is_alive() for i, p in enumerate(procs) if i not in out):
                break
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
            p.join()
    return out
