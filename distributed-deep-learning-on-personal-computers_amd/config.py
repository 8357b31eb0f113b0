"""Typed training configuration.

The reference keeps every knob as a module global or a literal:
``frequency_sending_gradients``/``batch_size``/``NN_in_model`` (ref.py:685-687),
``compress_model``/``model_bytes`` (ref.py:24-25), ``N_conn`` (ref.py:223), the
hard-coded server IP/port (ref.py:176-178), ``out_classes=6`` (ref.py:702), the
up-sample mode default (ref.py:621), 100 epochs (ref.py:720), 127 samples of 512²
(ref.py:737) and the last-30 test split (ref.py:672-673).

Here they are one dataclass, settable from a YAML/JSON file and from CLI flags.
Rendezvous is NOT part of the config: it comes from the torchrun environment
(RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, Optional

GRAD_CODECS = ("none", "fp16_absmax", "int8_absmax")
CODEC_SCALES = ("global", "bucket", "tensor")
REDUCE_OPS = ("mean", "sum", "reference")
UP_MODES = ("conv_transpose", "bilinear")
DATA_KINDS = ("synthetic", "vaihingen_dir")


@dataclass
class ModelConfig:
    """U-Net architecture knobs (ref.py:620-641)."""

    in_channels: int = 3
    out_classes: int = 6                 # ref.py:702
    width_divisor: int = 2               # NN_in_model, ref.py:687
    depth: int = 5                       # 5 levels in the reference; 4 for config #1
    up_sample_mode: str = "conv_transpose"  # ref.py:621
    dims: int = 2                        # 2 = images; 3 = volumes (BASELINE config #5)
    base_widths: tuple = (64, 128, 256, 512, 512)

    def widths(self):
        return [w // self.width_divisor for w in self.base_widths[: self.depth]]

    def validate(self):
        if self.up_sample_mode not in UP_MODES:
            raise ValueError(
                "Unsupported `up_sample_mode` (can take one of `conv_transpose` or `bilinear`)")
        if self.dims not in (2, 3):
            raise ValueError("dims must be 2 or 3")
        if not 1 <= self.depth <= len(self.base_widths):
            raise ValueError(f"depth must be in [1, {len(self.base_widths)}]")


@dataclass
class TrainConfig:
    model: ModelConfig = field(default_factory=ModelConfig)
    # ---- data ----------------------------------------------------------------
    data: str = "synthetic"              # synthetic | vaihingen_dir
    data_dir: Optional[str] = None       # directory of image + .npy label pairs (ref.py:660-674)
    tile: int = 256                      # H = W (D too for dims=3); reference: 512 (ref.py:737)
    num_samples: int = 127               # synthetic dataset length (ref.py:750: 127 tiles/epoch)
    test_holdout: int = 30               # last N pairs are the test split (ref.py:672-673)
    shard_data: bool = True              # False = reference "replicated data" mode (§2.2)
    shuffle: bool = True
    data_on_device: bool = True          # GPU: render / keep the dataset in HBM (K20)
    data_hbm_gb: Optional[float] = None  # HBM budget for a real dataset (None: half the free)
    # ---- optimisation ----------------------------------------------------------
    batch_per_gpu: int = 1               # batch_size, ref.py:686
    accum_steps: int = 1                 # frequency_sending_gradients, ref.py:685
    epochs: int = 1                      # reference: 100 (ref.py:720)
    max_steps: Optional[int] = None      # optimizer steps cap (benchmarks / smoke)
    lr: float = 1e-3                     # torch.optim.Adam defaults (ref.py:704)
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    dtype: str = "bf16"                  # compute dtype on GPU (fp32 master weights); "fp32"
                                         # (the reference's precision) = stock ops, no autocast
    seed: int = 0
    # ---- data parallel -----------------------------------------------------------
    backend: Optional[str] = None        # None = nccl(RCCL) on GPU, gloo on CPU
    bucket_mb: float = 8.0               # largest bucket (fp32 gradient MB)
    bucket_plan: str = "readiness"       # readiness: cuts placed by the backward readiness
                                         # model (parallel/bucket_plan.py) | size: size only
    reduce: str = "mean"                 # mean | sum | reference (the W=2 "sum" parity mode)
    grad_codec: str = "none"             # none | fp16_absmax | int8_absmax (ref.py:25)
    codec_scale: str = "bucket"          # global (reference parity) | bucket | tensor
    wire_dtype: str = "fp32"             # fp32 all-reduce | bf16 transport, fp32 accumulate
    overlap_comm: bool = True
    broadcast_buffers: bool = False      # BN running stats from rank 0 (reference: off)
    check_consistency_every: int = 0     # debug: all-reduce a param checksum every K steps
    reserve_cus: int = -1                # CUs kept out of persistent kernel grids so a
                                         # collective launched mid-backward starts at once
                                         # (-1 = auto = 0: measured, a bucket collective
                                         # starts within 20 us without it, and 8 reserved
                                         # CUs cost 5% of the step; docs/PERF.md)
    comm_proxy: int = 0                  # single GPU: stand-in collective for a world of N
                                         # (streaming kernel on a third stream, identity)
    timeout_s: int = 1800
    # fault injection: rank `fault_rank` exits (code 17) right after
    # optimizer step `fault_step`, on the first launch attempt only
    # (TORCHELASTIC_RESTART_COUNT == 0) — exercises torchrun --max-restarts + resume auto
    fault_rank: int = -1
    fault_step: int = 0
    # ---- io ----------------------------------------------------------------------
    ckpt_dir: Optional[str] = None
    ckpt_every: int = 0                  # optimizer steps; 0 = only at end of train()
    resume: Optional[str] = None
    log_dir: Optional[str] = None        # JSONL metrics + otus_<codec>.txt
    png_dir: Optional[str] = None        # prediction/label/image dumps (ref.py:785-790)
    png_count: int = 5
    log_every: int = 10
    # ---- tracing --------------------------------------------------
    trace_ranges: bool = False           # roctx ranges around the step phases
    phase_timers: bool = True            # hipEvent phase times (fwd+bwd, comm wait, optim)
    profile_dir: Optional[str] = None    # torch.profiler Chrome traces per rank
    profile_steps: int = 5               # active profiler steps (after 2 wait + 2 warm-up)
    # ---- execution -----------------------------------------------------------------
    impl: str = "auto"                   # auto | hip | torch   (hip = hand-written kernels, bf16;
                                         # auto = hip on a GPU for bf16, torch for fp32)
    hip_graph: bool = False              # capture the train step in a hipGraph
    micro_streams: int = -1              # accumulation micro-batches in flight on this many
                                         # HIP streams (each replaying its own graph); -1 =
                                         # auto: 3 for small accumulated micro-batches (the
                                         # reference's batch-1 regime), else 1 = one by one
    bn_window: int = -1                  # accumulation micro-batches run as ONE batched pass with
                                         # per-micro-batch BatchNorm groups (same math as the
                                         # micro-batches one by one: weights are fixed inside
                                         # the window, train-mode BN normalises per micro-batch):
                                         # 0 = off, k >= 2 = up to k micro-batches per pass,
                                         # -1 = auto (small accumulated micro-batches, HIP engine)
    recompute: int = 0                   # HIP engine activation recompute in backward (SURVEY 5.7,
                                         # batches beyond HBM): 1 = each block's first conv output,
                                         # 2 = both conv outputs of blocks that hand out a
                                         # materialised activation (+1 / +2 conv forwards)

    def validate(self):
        self.model.validate()
        for name, val, allowed in (("grad_codec", self.grad_codec, GRAD_CODECS),
                                   ("codec_scale", self.codec_scale, CODEC_SCALES),
                                   ("reduce", self.reduce, REDUCE_OPS),
                                   ("wire_dtype", self.wire_dtype, ("fp32", "bf16")),
                                   ("bucket_plan", self.bucket_plan, ("readiness", "size")),
                                   ("data", self.data, DATA_KINDS),
                                   ("impl", self.impl, ("auto", "hip", "torch")),
                                   ("dtype", self.dtype, ("bf16", "fp32"))):
            if val not in allowed:
                raise ValueError(f"{name}={val!r} not in {allowed}")
        if self.impl == "hip" and self.dtype != "bf16":
            # the hand-written kernels compute in bf16 (fp32 accumulation, fp32 master
            # weights); fp32 compute — the reference's precision (ref.py:702-704) — runs on
            # the stock-op path (impl="torch", or impl="auto" with dtype="fp32")
            raise ValueError("impl='hip' computes in bf16; use dtype='bf16', or impl='torch' / "
                             "'auto' for fp32 compute")
        if self.accum_steps < 1 or self.batch_per_gpu < 1:
            raise ValueError("accum_steps and batch_per_gpu must be >= 1")
        return self

    # ---- (de)serialisation ---------------------------------------------------------
    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d["model"]["base_widths"] = list(self.model.base_widths)
        d["betas"] = list(self.betas)
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "TrainConfig":
        d = dict(d)
        m = dict(d.pop("model", {}) or {})
        if "base_widths" in m:
            m["base_widths"] = tuple(m["base_widths"])
        known = {f.name for f in fields(cls)}
        unknown = set(d) - known
        if unknown:
            raise ValueError(f"unknown config keys: {sorted(unknown)}")
        if "betas" in d:
            d["betas"] = tuple(d["betas"])
        return cls(model=ModelConfig(**m), **d).validate()

    @classmethod
    def load(cls, path: str) -> "TrainConfig":
        with open(path) as f:
            if path.endswith((".yaml", ".yml")):
                import yaml
                d = yaml.safe_load(f)
            else:
                d = json.load(f)
        return cls.from_dict(d or {})

    def save(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2)


def _flag_type(tp, default):
    t = str(tp)                          # annotations are strings (postponed evaluation)
    if t in ("bool", "<class 'bool'>") or isinstance(default, bool):
        return lambda s: str(s).lower() in ("1", "true", "yes", "on")
    if isinstance(default, float) or t in ("float", "Optional[float]"):
        return float
    if isinstance(default, int) or t in ("int", "Optional[int]"):
        return lambda s: None if s in ("", "none", "None") else int(s)
    if isinstance(default, tuple):
        return lambda s: tuple(float(x) for x in s.split(","))
    return lambda s: None if s in ("", "none", "None") else s


def add_config_args(p: argparse.ArgumentParser):
    """Expose every TrainConfig/ModelConfig field as ``--name`` (model fields too)."""
    p.add_argument("--config", default=None, help="YAML/JSON config file")
    base = TrainConfig()
    for f in fields(TrainConfig):
        if f.name == "model":
            continue
        p.add_argument("--" + f.name.replace("_", "-"), dest=f.name, default=None,
                       type=_flag_type(f.type, getattr(base, f.name)))
    for f in fields(ModelConfig):
        if f.name == "base_widths":
            continue
        p.add_argument("--" + f.name.replace("_", "-"), dest="model__" + f.name, default=None,
                       type=_flag_type(f.type, getattr(base.model, f.name)))
    return p


def config_from_args(args: argparse.Namespace) -> TrainConfig:
    cfg = TrainConfig.load(args.config) if getattr(args, "config", None) else TrainConfig()
    for k, v in vars(args).items():
        if v is None or k == "config":
            continue
        if k.startswith("model__"):
            setattr(cfg.model, k[len("model__"):], v)
        elif hasattr(cfg, k):
            setattr(cfg, k, v)
    return cfg.validate()
