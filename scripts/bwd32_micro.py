#!/usr/bin/env python
"""Micro-benchmark of the fused 32-channel backward (conv3x3_bwd32.hip) against the two
kernels it replaces (resident data gradient with the BN-backward epilogue + v3 weight
gradient with the BN prologue) on the 256^2 x 32-channel level of the flagship U-Net."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from ddlpc.ops import _ext
    from ddlpc.ops.fused_unet import _ConvPack
    F = _ext.ops()
    dev = "cuda"
    N, H, C = a.batch, a.hw, 32
    y = (torch.randn(N, H, H, C, device=dev) * 1.3).bfloat16()
    dy = (torch.randn(N, H, H, C, device=dev) * 0.1).bfloat16()
    s4 = torch.stack([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev).contiguous()
    conv = torch.nn.Module()
    conv.weight = torch.nn.Parameter(torch.randn(C, C, 3, 3, device=dev) * 0.05)
    pk = _ConvPack(conv, 0, True)
    F.weight_pack(torch.tensor([pk.entry()], dtype=torch.int64, device=dev), 1, pk.numel())
    dw = torch.zeros(C, C, 3, 3, device=dev)

    def fused():
        F.conv3_bwd32(dy, y, s4, pk.dgrad, dw)

    def separate():
        F.conv3_fwd(dy, None, pk.dgrad, None, None, None, C, 0, False, None, None, y, s4)
        F.conv3_wgrad(dy, y, None, s4[2], s4[3], dw)

    def dgrad_only():
        F.conv3_fwd(dy, None, pk.dgrad, None, None, None, C, 0, False, None, None, y, s4)

    def wgrad_only():
        F.conv3_wgrad(dy, y, None, s4[2], s4[3], dw)

    T = N * H * H * C * 2
    for name, fn in (("fused", fused), ("separate", separate), ("dgrad_bnb", dgrad_only),
                     ("wgrad_pro", wgrad_only), ("fused", fused)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        print(f"{name:10s} {us:8.1f} us   ({3.27 * T / us / 1e3:6.0f} GB/s at 3.27 T)", flush=True)


if __name__ == "__main__":
    main()
