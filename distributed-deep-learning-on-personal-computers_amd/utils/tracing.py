"""Tracing / profiling hooks.

Reference: ``time.time()`` deltas printed around every phase (C25, e.g. ref.py:258,265,317,
388-389,440,760-770,778) with no device synchronisation, so GPU time is smeared into
whichever later call blocks.

Here:

* ``trace_range(name)`` — roctx ranges (``torch.cuda.nvtx`` is roctx on ROCm builds of
  PyTorch), visible in ``rocprofv3 --marker-trace`` and in ``torch.profiler`` traces;
  enabled by ``TrainConfig.trace_ranges`` or ``DDLPC_TRACE_RANGES=1``, free otherwise;
* ``PhaseTimer`` — hipEvents recorded on the compute stream at the phase boundaries of a
  train step (forward+backward, exposed gradient-communication wait, optimizer) and read
  lazily at log points (no per-step host sync);
* ``StepProfiler`` — ``torch.profiler`` with CPU + GPU (ROCm) activities over a window of
  steps, exporting a Chrome trace per rank.
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Dict, List, Optional

import torch

_RANGES = os.environ.get("DDLPC_TRACE_RANGES", "0") not in ("", "0")


def enable_ranges(on: bool = True):
    global _RANGES
    _RANGES = bool(on)


def ranges_enabled() -> bool:
    return _RANGES


@contextlib.contextmanager
def trace_range(name: str):
    """A roctx range around a host-side phase (no-op unless enabled or without a GPU)."""
    if not _RANGES or not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class PhaseTimer:
    """Per-step device phase times from hipEvents on the current (compute) stream.

    ``mark(name)`` records an event; the elapsed time between consecutive marks is that
    phase.  ``end_step()`` keeps the step's events; ``read()`` (call at log points, after
    something already synchronised) returns the mean ms per phase over the kept steps.
    On a CPU device (gloo rehearsal: every op and collective is synchronous on the host)
    the marks are host clock readings instead.
    """

    def __init__(self, device: torch.device, keep: int = 64):
        self.cuda = torch.device(device).type == "cuda"
        self.on = True
        self.keep = keep
        self._cur: List = []
        self._done: List[List] = []

    def mark(self, name: str):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
        else:
            e = time.perf_counter()
        self._cur.append((name, e))

    def end_step(self):
        if not self._cur:
            return
        self._done.append(self._cur)
        self._cur = []
        if len(self._done) > self.keep:
            self._done.pop(0)

    def _elapsed(self, a, b) -> float:
        return a.elapsed_time(b) if self.cuda else (b - a) * 1e3

    def read(self, reset: bool = True) -> Dict[str, float]:
        if not self._done:
            return {}
        tot: Dict[str, float] = {}
        n = 0
        for marks in self._done:
            if self.cuda and not marks[-1][1].query():
                continue
            n += 1
            for (_, a), (name, b) in zip(marks[:-1], marks[1:]):
                tot[name] = tot.get(name, 0.0) + self._elapsed(a, b)
            tot["step"] = tot.get("step", 0.0) + self._elapsed(marks[0][1], marks[-1][1])
        if reset:
            self._done = []
        return {f"{k}_ms": v / n for k, v in tot.items()} if n else {}


class StepProfiler:
    """``torch.profiler`` over steps [wait+warmup, wait+warmup+active) of a run; one Chrome
    trace per rank in ``out_dir`` (``trace_rank{r}.json``) plus a kernel table."""

    def __init__(self, out_dir: Optional[str], rank: int = 0, wait: int = 2, warmup: int = 2,
                 active: int = 5):
        self.prof = None
        if not out_dir:
            return
        from torch.profiler import ProfilerActivity, profile, schedule
        os.makedirs(out_dir, exist_ok=True)
        acts = [ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(ProfilerActivity.CUDA)      # ROCm/roctracer activities on ROCm

        def _ready(p):
            p.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))
            try:
                key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
                with open(os.path.join(out_dir, f"kernels_rank{rank}.txt"), "w") as f:
                    f.write(p.key_averages().table(sort_by=key, row_limit=60))
            except Exception:                       # table formatting is best-effort
                pass

        self.prof = profile(activities=acts, schedule=schedule(wait=wait, warmup=warmup,
                                                                 active=active, repeat=1),
                            on_trace_ready=_ready, record_shapes=False)
        self.prof.__enter__()

    def step(self):
        if self.prof is not None:
            self.prof.step()

    def close(self):
        if self.prof is not None:
            self.prof.__exit__(None, None, None)
            self.prof = None
