"""Command-line entry point: ``python -m ddlpc {train,validate,config}``.

The reference is started by hand on every PC (server first, then workers; rank from a
hostname table, ref.py:223-251) and has no flags at all.  Here one command
line serves every rank: launch it under ``torchrun`` (RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT come from the environment), e.g.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m ddlpc train \
        --batch-per-gpu 32 --accum-steps 1 --epochs 100 --log-dir runs/x

Every ``TrainConfig`` / ``ModelConfig`` field is a ``--flag`` (``--config file.yaml`` first,
flags override).  ``train`` prints the final reduced metrics as one JSON line on rank 0;
``validate`` evaluates a checkpoint on the held-out split; ``config`` prints the resolved
configuration (handy for writing a YAML to start from).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List, Optional

from .config import add_config_args, config_from_args


def _rank0() -> bool:
    return int(os.environ.get("RANK", "0")) == 0


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="ddlpc", description=__doc__.split("\n\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    p_train = add_config_args(sub.add_parser("train", help="train a U-Net (all ranks)"))
    p_train.add_argument("--device", default=None, help="cuda[:i] | cpu (default: auto)")
    p_val = add_config_args(sub.add_parser("validate", help="evaluate on the held-out split"))
    p_val.add_argument("--checkpoint", default=None)
    p_val.add_argument("--device", default=None)
    add_config_args(sub.add_parser("config", help="print the resolved config as JSON"))
    args = ap.parse_args(argv)
    cmd = args.cmd
    device = getattr(args, "device", None)
    checkpoint = getattr(args, "checkpoint", None)
    for k in ("cmd", "device", "checkpoint"):
        if hasattr(args, k):
            delattr(args, k)
    cfg = config_from_args(args)
    if cmd == "config":
        print(json.dumps(cfg.to_dict(), indent=2))
        return 0
    from .train.trainer import train, validate
    if cmd == "train":
        metrics = train(cfg, device=device)
    else:
        metrics = validate(cfg, checkpoint=checkpoint, device=device)
    if _rank0():
        print(json.dumps({"cmd": cmd, **{k: (float(v) if isinstance(v, (int, float)) else v)
                                         for k, v in (metrics or {}).items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
