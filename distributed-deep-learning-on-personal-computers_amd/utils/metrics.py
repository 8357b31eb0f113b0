"""Metrics, run logs, timers and visual dumps (C23-C25).

Reference: per-iteration pixel accuracy and loss read back to the host on rank 0 every
micro-batch (ref.py:775-777), an ``otus_{model_bytes}.txt`` log with a header and one line
per epoch (ref.py:715-716,781-782), ``time.time()`` deltas without device sync (C25), and
5 PNG triplets per epoch (ref.py:785-790).

Here: device-side accumulators (no per-step host sync), cross-rank reduction at log time,
a JSONL stream, an ``otus_<codec>.txt``-compatible writer, hipEvent step timers, and the
PNG dump as a callback under ``no_grad`` + ``eval`` (the reference runs it in train mode,
updating BN statistics).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist


_HIP = False


def _hip_ops():
    """``torch.ops.ddlpc`` when the kernel library is built, else None (CPU runs)."""
    global _HIP
    if _HIP is False:
        from ..ops import _ext
        _HIP = _ext.ops() if _ext.load(strict=False) else None
    return _HIP


class DeviceMeter:
    """Accumulates loss*n, correct pixels, pixel count on the device."""

    def __init__(self, device):
        self.device = device
        self.reset()

    def reset(self):
        # in place once allocated: a captured train step (hipGraph) keeps accumulating into
        # the same buffer
        if getattr(self, "buf", None) is None:
            self.buf = torch.zeros(4, dtype=torch.float64, device=self.device)
            self._inc_pixels = None
            self._inc = None
        else:
            self.buf.zero_()

    def add(self, loss: torch.Tensor, correct: torch.Tensor, pixels: int, n: int = 1):
        # [sum loss, sum correct, sum pixels, micro-batches]; no host->device copies per step.
        # n > 1: a batched window of n micro-batches whose mean per-micro-batch loss is `loss`
        if (loss.dtype == torch.float32 and correct.dtype == torch.float32
                and loss.numel() == 1 and correct.numel() == 1 and _hip_ops() is not None):
            # one launch instead of five small elementwise kernels
            _hip_ops().meter_add(self.buf, loss.detach(), correct.detach(), float(pixels), float(n))
            return
        if self._inc_pixels != (pixels, n):
            self._inc = torch.tensor([float(pixels), float(n)], dtype=torch.float64,
                                     device=self.device)
            self._inc_pixels = (pixels, n)
        self.buf[:2] += torch.stack([loss.detach().double() * n, correct.detach().double()])
        self.buf[2:] += self._inc

    def reduce(self, group=None) -> Dict[str, float]:
        b = self.buf.clone()
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(b, group=group)
        s = b.cpu().tolist()
        n = max(s[3], 1.0)
        return {"loss": s[0] / n, "pixel_acc": s[1] / max(s[2], 1.0), "micro_batches": s[3]}


class StepTimer:
    """hipEvent-based (CUDA API) timer; falls back to perf_counter on CPU."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"
        self.t0 = self.e0 = None

    def start(self):
        if self.cuda:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        self.t0 = time.perf_counter()

    def stop_ms(self) -> float:
        if self.cuda:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            e1.synchronize()
            return self.e0.elapsed_time(e1)
        return (time.perf_counter() - self.t0) * 1e3


class RunLogger:
    def __init__(self, log_dir: Optional[str], rank: int = 0, codec: str = "none"):
        self.rank, self.log_dir = rank, log_dir
        self.jsonl = self.otus = None
        if log_dir and rank == 0:
            os.makedirs(log_dir, exist_ok=True)
            self.jsonl = open(os.path.join(log_dir, "metrics.jsonl"), "a")
            name = {"none": "float32", "fp16_absmax": "float16", "int8_absmax": "int8"}[codec]
            self.otus_path = os.path.join(log_dir, f"otus_{name}.txt")

    def header(self, batch_per_gpu: int, world: int, accum: int, width_divisor: int):
        """ref.py:716 header (its "total batch" ignores accumulation; we keep that)."""
        if self.rank != 0 or not self.log_dir:
            return
        with open(self.otus_path, "w") as f:
            f.write(" ".join(map(str, [
                "\nbatch_size на одном ПК:", batch_per_gpu,
                "\nОбщий размер batch_size (все ПК):", batch_per_gpu * world,
                "\nЧастота передачи данных (градиентов):", accum,
                "\nделитель размер сети:", width_divisor,
                "\nколичество ПК (включая сервер)", world, "\n\n"])))

    def epoch_line(self, ep: int, mean_loss: float, mean_acc: float, epoch_s: float,
                   per_sync_s: float):
        """ref.py:782 per-epoch line."""
        if self.rank != 0 or not self.log_dir:
            return
        with open(self.otus_path, "a") as f:
            f.write(" ".join(map(str, [
                "\nep:", ep, "mean_loss", mean_loss, "mean_accuracy", mean_acc,
                "время на все примеры эпохи", epoch_s, "общее время", epoch_s,
                "среднее время на батч:", per_sync_s, "\n"])))

    def log(self, rec: dict):
        if self.jsonl is not None:
            self.jsonl.write(json.dumps(rec) + "\n")
            self.jsonl.flush()

    def close(self):
        if self.jsonl is not None:
            self.jsonl.close()
            self.jsonl = None


def iou_per_class(pred: torch.Tensor, target: torch.Tensor, classes: int) -> torch.Tensor:
    """Per-class intersection-over-union counts -> IoU (nan for absent classes)."""
    p = pred.reshape(-1)
    t = target.reshape(-1)
    idx = t * classes + p
    cm = torch.bincount(idx, minlength=classes * classes).reshape(classes, classes).double()
    inter = cm.diag()
    union = cm.sum(0) + cm.sum(1) - inter
    iou = inter / union.clamp_min(1)
    iou[union == 0] = float("nan")
    return iou


def confusion_matrix(pred: torch.Tensor, target: torch.Tensor, classes: int) -> torch.Tensor:
    idx = target.reshape(-1) * classes + pred.reshape(-1)
    return torch.bincount(idx, minlength=classes * classes).reshape(classes, classes)


@torch.no_grad()
def dump_pngs(model, x: torch.Tensor, y: torch.Tensor, out_dir: str, count: int = 5):
    """``Model {i}.png`` (argmax*5), ``Label {i}.png`` (label*5), ``Image {i}.png``
    (ref.py:785-790), in eval mode without building graphs."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from PIL import Image
    os.makedirs(out_dir, exist_ok=True)
    was_training = model.training
    model.eval()
    try:
        for i in range(min(count, x.shape[0])):
            xi = x[i:i + 1]
            out = model(xi).float().argmax(1)[0].cpu().numpy()
            plt.imsave(os.path.join(out_dir, f"Model {i}.png"), np.uint8(out * 5))
            plt.imsave(os.path.join(out_dir, f"Label {i}.png"),
                       np.uint8(y[i].cpu().numpy() * 5))
            img = xi[0].float().cpu().numpy().transpose(1, 2, 0)
            Image.fromarray(np.uint8(np.clip(img, 0, 1) * 255)).save(
                os.path.join(out_dir, f"Image {i}.png"))
    finally:
        model.train(was_training)
