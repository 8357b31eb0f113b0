"""Checkpoint save / resume.

The reference has NO checkpointing: its only model serialisation is the
pickled ``[UNet, Adam, CrossEntropyLoss]`` wire message of the initial broadcast
(ref.py:561).  This module adds:

* ``torch.save({"model", "optimizer", "epoch", "step", "micro_step", "epoch_step", "config",
  "rng"})`` (``epoch_step``: optimizer steps done in ``epoch``, so a resume continues mid-epoch);
* ``model`` is the standard ``state_dict`` with the reference's exact 166 keys
  (``down_conv{1..5}.double_conv.double_conv.{0,1,3,4}.*``, ``double_conv.double_conv.*``,
  ``up_conv{5..1}.up_sample.*``, ``up_conv{k}.double_conv.double_conv.*``,
  ``conv_last.*``) in standard PyTorch layouts (OIHW conv, IOHW transposed conv, fp32) —
  internal bf16/NHWC kernel copies are never saved;
* ``optimizer`` is ``torch.optim.Adam``-format (loads into stock Adam and vice versa);
* loading uses ``torch.load(weights_only=True)``: nothing in a checkpoint is executed.

Files are written atomically (tmp + rename) by rank 0 only.
"""
from __future__ import annotations

import os
import re
from typing import Any, Dict, Optional

import torch


def rng_state() -> Dict[str, Any]:
    st = {"torch": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: Dict[str, Any]):
    if "torch" in st:
        torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def save_checkpoint(path: str, model: torch.nn.Module, optimizer=None, epoch: int = 0,
                    step: int = 0, micro_step: int = 0, config: Optional[dict] = None,
                    extra: Optional[dict] = None, epoch_step: int = 0):
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    sd = {k: v.detach().cpu() if torch.is_tensor(v) else v
          for k, v in model.state_dict().items()}
    blob = {"model": sd, "epoch": int(epoch), "step": int(step), "micro_step": int(micro_step),
            "epoch_step": int(epoch_step),
            "config": config or {}, "rng": rng_state(), "format": "ddlpc-ckpt-v1"}
    if optimizer is not None:
        osd = optimizer.state_dict()
        osd["state"] = {k: {n: (t.detach().cpu().clone() if torch.is_tensor(t) else t)
                            for n, t in v.items()} for k, v in osd["state"].items()}
        blob["optimizer"] = osd
    if extra:
        blob["extra"] = extra
    tmp = path + ".tmp"
    torch.save(blob, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, model: Optional[torch.nn.Module] = None, optimizer=None,
                    map_location="cpu", restore_rng: bool = True) -> Dict[str, Any]:
    blob = torch.load(path, map_location=map_location, weights_only=True)
    if model is not None:
        sd = blob["model"] if "model" in blob else blob     # bare state_dict also accepted
        with torch.no_grad():
            own = model.state_dict()
            missing = set(own) - set(sd)
            unexpected = set(sd) - set(own)
            if missing or unexpected:
                raise KeyError(f"state_dict mismatch: missing={sorted(missing)[:5]} "
                               f"unexpected={sorted(unexpected)[:5]}")
            for k, v in sd.items():
                own[k].copy_(v)                     # in place: keeps flat-buffer views
    if optimizer is not None and "optimizer" in blob:
        optimizer.load_state_dict(blob["optimizer"])
    if restore_rng and "rng" in blob:
        set_rng_state(blob["rng"])
    return blob


def latest_checkpoint(ckpt_dir: str) -> Optional[str]:
    if not ckpt_dir or not os.path.isdir(ckpt_dir):
        return None
    # only the step-numbered files Trainer.save() writes (ckpt_final.pt etc. are ignored)
    cands = [(int(m.group(1)), f) for f in os.listdir(ckpt_dir)
             for m in [re.fullmatch(r"ckpt_(\d+)\.pt", f)] if m]
    if not cands:
        return None
    return os.path.join(ckpt_dir, max(cands)[1])
