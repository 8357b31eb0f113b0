"""Process-group rendezvous and initial state broadcast.

Reference: a hard-coded server IP:port (ref.py:176-178,195-201),
a static hostname->rank dictionary (ref.py:226-251), blocking TCP accept of exactly
``N_conn`` workers (ref.py:184-189), then rank 0 pickles the LIVE ``[model, optimizer,
criterion]`` objects to every worker (ref.py:560-565, ref.py:708/810).

Here: torchrun's environment rendezvous (``RANK``, ``WORLD_SIZE``, ``LOCAL_RANK``,
``MASTER_ADDR``/``MASTER_PORT``) into ``torch.distributed`` — backend ``nccl`` (= RCCL on
ROCm, over xGMI inside a node, RoCE/TCP across nodes: the "personal computers over a
LAN" capability) or ``gloo`` on CPU.  Every rank builds its own model and optimizer from
the shared config and seed; rank 0's parameters and buffers are then broadcast as ONE
coalesced flat buffer per dtype (no pickles cross the wire, nothing is unpickled).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: Optional[str] = None
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


def env_info() -> DistInfo:
    return DistInfo(rank=int(os.environ.get("RANK", 0)),
                    world_size=int(os.environ.get("WORLD_SIZE", 1)),
                    local_rank=int(os.environ.get("LOCAL_RANK", 0)))


def init_distributed(backend: Optional[str] = None, timeout_s: int = 1800,
                     device: Optional[str] = None) -> DistInfo:
    """Initialise from the torchrun env.  Safe to call when WORLD_SIZE is 1 / unset.

    ``device``: "cuda" / "cpu" / None (cuda if available).  Picks ``nccl`` (RCCL) for GPU
    ranks and ``gloo`` otherwise unless ``backend`` is given.
    """
    info = env_info()
    use_cuda = (device == "cuda") or (device is None and torch.cuda.is_available())
    if use_cuda:
        torch.cuda.set_device(info.local_rank)
        info.device = torch.device("cuda", info.local_rank)
    else:
        info.device = torch.device("cpu")
    info.backend = backend or ("nccl" if use_cuda else "gloo")
    if info.world_size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # Asynchronous error handling so a dead peer aborts instead of hanging forever
        # (the reference's blocking sockets hang: SURVEY.md §5.3).
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=info.backend, rank=info.rank, world_size=info.world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if info.backend == "nccl":
            kw["device_id"] = info.device
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        if attempt != "0" and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
            # a torchrun restart (--max-restarts): the agent's store still holds the failed
            # attempt's keys, and gloo's full-mesh connect reads the dead peers' addresses
            # from them (connection refused).  Rendezvous under a per-attempt prefix.
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]),
                                 info.world_size, False,
                                 timeout=datetime.timedelta(seconds=timeout_s))
            kw["store"] = dist.PrefixStore(f"ddlpc/attempt_{attempt}", base)
        dist.init_process_group(**kw)
    elif dist.is_initialized():
        info.rank, info.world_size = dist.get_rank(), dist.get_world_size()
        info.backend = dist.get_backend()
    return info


def shutdown():
    if dist.is_initialized():
        try:
            dist.barrier()
        finally:
            dist.destroy_process_group()


def _coalesced_broadcast(tensors: List[torch.Tensor], src: int, group=None):
    """Broadcast a list of tensors as one flat buffer per dtype (one collective each)."""
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dtype, ts in by_dtype.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


def broadcast_module(module: torch.nn.Module, src: int = 0, group=None,
                     buffers: bool = True):
    """Rank ``src`` -> all: parameters (+ buffers).  Replaces ref.py:560-565."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    ts = [p.data for p in module.parameters()]
    if buffers:
        ts += [b for b in module.buffers()]
    _coalesced_broadcast(ts, src, group)


def broadcast_buffers(module: torch.nn.Module, src: int = 0, group=None):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    bufs = [b for b in module.buffers()]
    if bufs:
        _coalesced_broadcast(bufs, src, group)


def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0, group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return
    _coalesced_broadcast(list(tensors), src, group)


def params_checksum(module: torch.nn.Module) -> torch.Tensor:
    """Order-sensitive float64 checksum of all parameters (race/desync detector)."""
    acc = None
    for i, p in enumerate(module.parameters()):
        v = p.detach().double().sum() * (1.0 + 1e-3 * (i % 97)) + p.detach().double().abs().sum()
        acc = v if acc is None else acc + v
    return acc if acc is not None else torch.zeros((), dtype=torch.float64)


def assert_replicas_identical(module: torch.nn.Module, group=None, tol: float = 0.0):
    """Debug mode: all-reduce MAX/MIN of a parameter checksum and raise
    if ranks diverged.  ``tol`` = 0 demands bit-identical replicas."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    c = params_checksum(module)
    dev = next(module.parameters()).device
    hi = c.clone().to(dev)
    lo = c.clone().to(dev)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    if float(hi - lo) > tol * max(1.0, abs(float(hi))):
        raise RuntimeError(f"replica divergence: checksum spread {float(hi - lo)!r}")
