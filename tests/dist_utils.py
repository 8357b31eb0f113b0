"""Spawn a gloo "fake cluster" on localhost (the reference needs 6 named PCs;
this runs the same data-parallel protocol in W processes on 127.0.0.1)."""
import os
import traceback

import torch.multiprocessing as mp


def _agent_store(world):
    """The rendezvous store, hosted by the test process the way torchrun's agent hosts it:
    bound to port 0 by the store itself (no probe-then-bind race with other processes) and
    kept open for the run; every rank connects to it as a client
    (TORCHELASTIC_USE_AGENT_STORE)."""
    import datetime

    import torch.distributed as dist
    return dist.TCPStore("127.0.0.1", 0, world, True, timeout=datetime.timedelta(seconds=300),
                         wait_for_workers=False)


def _entry(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      TORCHELASTIC_USE_AGENT_STORE="True", TORCHELASTIC_RESTART_COUNT="0")
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


def run(fn, world=2, args=(), timeout=240, allow_fail=False):
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
    store = _agent_store(world)          # (kept alive until every rank has finished)
    port = store.port
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
    del store
    return out
