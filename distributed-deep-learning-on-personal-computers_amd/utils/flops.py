"""Model-geometry FLOP counts for the roofline fields of ``bench.py``.

The U-Net's work is its convolutions (22 conv3x3, 5 transposed convs, the
1x1 head; BN/ReLU/pool are O(activations)).  Forward multiply-accumulates are counted by
forward hooks on the stock ``nn`` model at a small probe tile and scaled by the pixel ratio
(every conv's MACs are linear in the pixel count).  A training step is counted as
3 x forward (forward + data gradient + weight gradient), the convention of SURVEY.md §2.5
(85.0 GFLOP per 256² image at width divisor 2).
"""
from __future__ import annotations

import functools

import torch
import torch.nn as nn

# MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md, chip-level parameters; no sparsity)
PEAK_BF16_TFLOPS = 2500.0


@functools.lru_cache(maxsize=None)
def _forward_macs_probe(in_channels: int, out_classes: int, width_divisor: int, depth: int,
                        up_sample_mode: str, dims: int, probe: int) -> int:
    from ..config import ModelConfig
    from ..models.unet import UNet
    cfg = ModelConfig(in_channels=in_channels, out_classes=out_classes,
                      width_divisor=width_divisor, depth=depth,
                      up_sample_mode=up_sample_mode, dims=dims)
    with torch.device("meta"):
        model = UNet.from_config(cfg)
    total = [0]

    def hook(mod, inp, out):
        if isinstance(mod, (nn.Conv2d, nn.Conv3d)):
            k = 1
            for s in mod.kernel_size:
                k *= s
            total[0] += out.numel() * (mod.in_channels // mod.groups) * k
        elif isinstance(mod, (nn.ConvTranspose2d, nn.ConvTranspose3d)):
            # stride == kernel: every output element is one Cin-long dot product
            total[0] += out.numel() * mod.in_channels

    hs = [m.register_forward_hook(hook) for m in model.modules()
          if isinstance(m, (nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.ConvTranspose3d))]
    shape = (1, in_channels) + (probe,) * dims
    with torch.no_grad():
        model(torch.empty(shape, device="meta"))
    for h in hs:
        h.remove()
    return total[0]


def unet_train_flops_per_sample(model_cfg, tile: int) -> float:
    """Training FLOPs (3 x forward, 2 FLOP per MAC) for ONE image / volume of edge ``tile``."""
    probe = 2 ** model_cfg.depth * 2          # smallest tile every level divides
    macs = _forward_macs_probe(model_cfg.in_channels, model_cfg.out_classes,
                               model_cfg.width_divisor, model_cfg.depth,
                               model_cfg.up_sample_mode, model_cfg.dims, probe)
    scale = (tile / probe) ** model_cfg.dims
    return 3.0 * 2.0 * macs * scale


@functools.lru_cache(maxsize=None)
def _activation_elems_probe(in_channels: int, out_classes: int, width_divisor: int, depth: int,
                            up_sample_mode: str, dims: int, probe: int) -> int:
    from ..config import ModelConfig
    from ..models.unet import UNet
    cfg = ModelConfig(in_channels=in_channels, out_classes=out_classes,
                      width_divisor=width_divisor, depth=depth,
                      up_sample_mode=up_sample_mode, dims=dims)
    with torch.device("meta"):
        model = UNet.from_config(cfg)
    total = [0]
    kinds = (nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.ConvTranspose3d,
             nn.BatchNorm2d, nn.BatchNorm3d)

    def hook(mod, inp, out):
        total[0] += out.numel()

    hs = [m.register_forward_hook(hook) for m in model.modules() if isinstance(m, kinds)]
    with torch.no_grad():
        model(torch.empty((1, in_channels) + (probe,) * dims, device="meta"))
    for h in hs:
        h.remove()
    return total[0]


def unet_activation_elems_per_sample(model_cfg, tile: int) -> float:
    """Summed conv / transposed-conv / BatchNorm output elements of ONE sample at edge
    ``tile`` (every saved pre-BN and post-BN activation of a training step; SURVEY.md §2.5:
    ~228 M at 512² for width divisor 2) — the per-sample activation-memory yardstick."""
    probe = 2 ** model_cfg.depth * 2
    n = _activation_elems_probe(model_cfg.in_channels, model_cfg.out_classes,
                                model_cfg.width_divisor, model_cfg.depth,
                                model_cfg.up_sample_mode, model_cfg.dims, probe)
    return n * (tile / probe) ** model_cfg.dims
